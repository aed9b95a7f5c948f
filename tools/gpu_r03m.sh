# round 3 evidence in one call: smoke, the whole GPU parity suite, the default bench, the bench
# under the driver's arguments, then rocprofv3 kernel trace + FETCH/WRITE PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
rocm-smi --showclocks --showpower --showuse > gpurun_out/rocm_smi.txt 2>&1 || true
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 3
bash tools/gpu_profile.sh || exit 4
echo done
