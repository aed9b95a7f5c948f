# round 3 (session 2): one-launch TESA (table + scan per workgroup): parity, then A/B against the two-launch form
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tesa.py tests/test_gpu_4k.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ad_pytest.log 2>&1 || { tail -30 gpurun_out/r03ad_pytest.log; exit 1; }
tail -2 gpurun_out/r03ad_pytest.log
timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03ad_tesa_fused.log 2>&1 || exit 2
X264HIP_TESA_VARIANT=3 timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03ad_tesa_two.log 2>&1 || exit 3
timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03ad_tesa_fused2.log 2>&1 || exit 4
cat gpurun_out/r03ad_tesa_fused.log gpurun_out/r03ad_tesa_two.log gpurun_out/r03ad_tesa_fused2.log
