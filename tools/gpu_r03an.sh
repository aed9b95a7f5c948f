# round 3 (session 2) evidence of the final tree: full GPU suite + smoke, default bench, kernel trace + stats, FETCH / WRITE PMC, then the driver-argument bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03an_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03an_pytest_gpu.log; exit 6; }
tail -2 gpurun_out/r03an_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03an_smoke.log 2>&1 || { tail -20 gpurun_out/r03an_smoke.log; exit 7; }
rocm-smi --showclocks --showpower --showuse > gpurun_out/rocm_smi.txt 2>&1 || true
bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 5
echo done
