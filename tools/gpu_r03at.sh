# round 3 (session 2): the final in-tree library: smoke + TESA / DCT / runtime parity
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03at_smoke.log 2>&1 || { tail -20 gpurun_out/r03at_smoke.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_tesa.py tests/test_gpu_dct.py tests/test_gpu_runtime.py tests/test_gpu_me.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03at_pytest.log 2>&1 || { tail -30 gpurun_out/r03at_pytest.log; exit 2; }
tail -1 gpurun_out/r03at_pytest.log
