# round 3, first GPU call: the new runtime / lookahead / ESA-range tests, the host-link
# probe, the bench under the driver's arguments (1 rank, then 2 gloo ranks sharing the GPU
# with no launcher, then --gpus 8 which must be refused), and a kernel trace of the bench
# under the driver's arguments (hpel_filter event time vs kernel time)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_lookahead.py tests/test_gpu_me.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/link_probe.py gpurun_out/r03a_link_probe.json > gpurun_out/r03a_link_probe.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03a_bench_driver.log 2>&1 || exit 3
X264HIP_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r03a_bench_gloo2.log 2>&1 || exit 4
timeout -k 10 100 python bench.py --gpus 8 > gpurun_out/r03a_bench_gpus8.log 2>&1; echo "rc=$?" >> gpurun_out/r03a_bench_gpus8.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03a_trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $R/gpurun_out/r03a_trace.log 2>&1 || exit 5
echo done
