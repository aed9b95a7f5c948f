# round 3 call b: streaming-leg A/B (tools/stream_probe.py) and the bench with 64-pair steps
# and graph-timed side legs under the driver's arguments
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_me_bind.py tests/test_gpu_lookahead.py tests/test_gpu_runtime.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/stream_probe.py gpurun_out/r03b_stream_probe.json > gpurun_out/r03b_stream_probe.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03b_bench_driver.log 2>&1 || exit 2
echo done
