set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/r03n_queues.log
for K in 0 1 2 3 4 5; do
  timeout -k 10 120 python tools/stream_queues.py $K 2>/dev/null | tail -1 >> gpurun_out/r03n_queues.log || exit 1
done
for K in 0 3; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/stream_queues.py $K 2>/dev/null | tail -1 >> gpurun_out/r03n_queues.log || exit 2
done
echo done
