# round 3: hpel variant 7 (slot reuse, buffer stores, 4 waves) parity + A/B against variant 3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mc.py tests/test_gpu_4k.py -k "hpel" > gpurun_out/r03t_pytest.log 2>&1 || { tail -30 gpurun_out/r03t_pytest.log; exit 1; }
tail -3 gpurun_out/r03t_pytest.log
timeout -k 10 400 python -u tools/stream_var_ab.py gpurun_out/r03t_stream_var.json > gpurun_out/r03t_stream_var.log 2>&1 || { tail -20 gpurun_out/r03t_stream_var.log; exit 1; }
cat gpurun_out/r03t_stream_var.json
