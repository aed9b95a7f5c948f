# round 3: full GPU suite with line-aligned hpel strips + nontemporal stores by default, A/Bs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03w_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03w_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03w_pytest_gpu.log
timeout -k 10 400 python -u tools/stream_var_ab.py gpurun_out/r03w_stream_var.json > gpurun_out/r03w_stream_var.log 2>&1 || { tail -20 gpurun_out/r03w_stream_var.log; exit 1; }
cat gpurun_out/r03w_stream_var.json
timeout -k 10 400 python -u tools/nt_ab.py gpurun_out/r03w_nt_ab.json > gpurun_out/r03w_nt_ab.log 2>&1 || { tail -20 gpurun_out/r03w_nt_ab.log; exit 1; }
cat gpurun_out/r03w_nt_ab.json
