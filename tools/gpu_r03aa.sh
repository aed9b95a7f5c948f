# round 3: plane SSD with one packed atomic per workgroup: parity + A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ssd_plane.py > gpurun_out/r03aa_pytest.log 2>&1 || { tail -30 gpurun_out/r03aa_pytest.log; exit 1; }
tail -2 gpurun_out/r03aa_pytest.log
timeout -k 10 300 python -u tools/ssd_ab.py gpurun_out/r03aa_ssd_ab.json > gpurun_out/r03aa_ssd_ab.log 2>&1 || { tail -20 gpurun_out/r03aa_ssd_ab.log; exit 1; }
cat gpurun_out/r03aa_ssd_ab.json
