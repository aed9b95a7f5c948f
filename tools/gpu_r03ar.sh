# round 3 (session 2): runtime tests (empty launches, TESA stride refusal)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ar_pytest.log 2>&1 || { tail -30 gpurun_out/r03ar_pytest.log; exit 1; }
tail -2 gpurun_out/r03ar_pytest.log
