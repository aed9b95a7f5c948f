# round 3 (session 2): bench.py JSON contract test on the GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -q --timeout 350 --timeout-method thread > gpurun_out/r03am_pytest.log 2>&1 || { tail -40 gpurun_out/r03am_pytest.log; exit 1; }
tail -2 gpurun_out/r03am_pytest.log
