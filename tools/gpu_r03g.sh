set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssd_plane.py tests/test_gpu_pixel.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g_pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/ssd_time.py > gpurun_out/r03g_ssd.log 2>&1 || exit 2
echo done
