# round 3 call d: XCD remap default (ME parity tests), bench driver args + 2160p host timing
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_me.py tests/test_gpu_4k.py tests/test_gpu_tesa.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03d_bench_driver.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --no-cpu > gpurun_out/r03d_bench_100.log 2>&1 || exit 3
echo done
