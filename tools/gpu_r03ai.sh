# round 3 (session 2): full GPU suite + smoke of the tree with the sector-shifted DCT strips and the one-launch TESA variant
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ai_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03ai_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03ai_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ai_smoke.log 2>&1 || { tail -20 gpurun_out/r03ai_smoke.log; exit 2; }
tail -1 gpurun_out/r03ai_smoke.log
