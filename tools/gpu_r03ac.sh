# round 3 (session 2): full GPU suite, smoke and the driver-argument bench of the rebuilt tree
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ac_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03ac_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03ac_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ac_smoke.log 2>&1 || { tail -20 gpurun_out/r03ac_smoke.log; exit 2; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03ac_bench_driver.log 2>&1 || { tail -20 gpurun_out/r03ac_bench_driver.log; exit 3; }
tail -c 3000 gpurun_out/r03ac_bench_driver.log
