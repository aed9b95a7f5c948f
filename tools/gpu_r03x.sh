# round 3: plane SSD rows-per-wave A/B + kernel trace of the 16-frame leg
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ssd_plane.py > gpurun_out/r03x_pytest.log 2>&1 || { tail -30 gpurun_out/r03x_pytest.log; exit 1; }
tail -2 gpurun_out/r03x_pytest.log
timeout -k 10 300 python -u tools/ssd_ab.py gpurun_out/r03x_ssd_ab.json > gpurun_out/r03x_ssd_ab.log 2>&1 || { tail -20 gpurun_out/r03x_ssd_ab.log; exit 1; }
cat gpurun_out/r03x_ssd_ab.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03x_tr -o run -- python3 $R/tools/ssd_time.py > $R/gpurun_out/r03x_tr.log 2>&1 || exit 3
find $R/gpurun_out/r03x_tr -name '*kernel_stats.csv' -exec grep -i ssd {} \;
