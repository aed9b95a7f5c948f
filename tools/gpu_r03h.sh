set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/stream_xcd_ab.py gpurun_out/r03h_stream_xcd.json > gpurun_out/r03h_stream_xcd.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_pytest.log 2>&1 || exit 2
echo done
