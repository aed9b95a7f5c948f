# upload entry: runtime GPU tests, then the bench (2160p streaming legs: SDMA copy vs upload kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_runtime.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_upload.log 2>&1 || exit 2
echo done
