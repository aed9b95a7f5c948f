# round 3 call f: TESA speculative scans (parity + A/B), plane SSD ticket finish (parity + time)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tesa.py tests/test_gpu_ssd_plane.py tests/test_gpu_4k.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03f_tesa_spec.log 2>&1 || exit 2
X264HIP_TESA_VARIANT=2 timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03f_tesa_chain.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03f_bench_driver.log 2>&1 || exit 4
echo done
