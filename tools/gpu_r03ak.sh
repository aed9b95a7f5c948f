# round 3 (session 2): 10-bit 8x8 DCT default = one-wave staged strips (variant 11): parity, then the driver-argument bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dct.py tests/test_gpu_4k.py tests/test_gpu_runtime.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ak_pytest.log 2>&1 || { tail -30 gpurun_out/r03ak_pytest.log; exit 1; }
tail -2 gpurun_out/r03ak_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03ak_bench_driver.log 2>&1 || { tail -20 gpurun_out/r03ak_bench_driver.log; exit 2; }
tail -c 1500 gpurun_out/r03ak_bench_driver.log
