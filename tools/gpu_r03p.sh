set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/r03p_after.log
for Q in 4 8 16; do
  for L in ssd tesa; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 150 python tools/stream_after.py $L 2>/dev/null | tail -1 | sed "s/^{/{\"queues\": $Q, /" >> gpurun_out/r03p_after.log || exit 1
  done
done
echo done
