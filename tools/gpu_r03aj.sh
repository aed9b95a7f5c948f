# round 3 (session 2): staged strip DCT with nontemporal stores / one-wave workgroups (variants 11, 12): parity + A/B at 8 and 10 bit, then the full GPU suite and smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dct.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aj_pytest.log 2>&1 || { tail -30 gpurun_out/r03aj_pytest.log; exit 1; }
tail -2 gpurun_out/r03aj_pytest.log
DQ_BD=10 timeout -k 10 300 python tools/dq_time.py > gpurun_out/r03aj_dq_ab10.log 2>&1 || { tail gpurun_out/r03aj_dq_ab10.log; exit 2; }
tail -1 gpurun_out/r03aj_dq_ab10.log
timeout -k 10 300 python tools/dq_time.py > gpurun_out/r03aj_dq_ab8.log 2>&1 || { tail gpurun_out/r03aj_dq_ab8.log; exit 3; }
tail -1 gpurun_out/r03aj_dq_ab8.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aj_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03aj_pytest_gpu.log; exit 4; }
tail -2 gpurun_out/r03aj_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03aj_smoke.log 2>&1 || { tail -20 gpurun_out/r03aj_smoke.log; exit 5; }
tail -1 gpurun_out/r03aj_smoke.log
