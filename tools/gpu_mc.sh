set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_mc.py -x -q > gpurun_out/pytest_mc.log 2>&1
rc=$?; echo "pytest exit: $rc" >> gpurun_out/pytest_mc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench.log 2>&1
