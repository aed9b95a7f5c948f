set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/r03o_after.log
for L in none ssd hpel tesa esa lowres; do
  timeout -k 10 150 python tools/stream_after.py $L 2>/dev/null | tail -1 >> gpurun_out/r03o_after.log || exit 1
done
echo done
