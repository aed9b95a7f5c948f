# round 3: nontemporal-store A/B at the bench shapes + parity of the NT paths
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mc.py tests/test_gpu_dct.py -k "hpel_filter or lowres or mb_dct_quant_1080p" > gpurun_out/r03s_pytest.log 2>&1 || { tail -30 gpurun_out/r03s_pytest.log; exit 1; }
tail -3 gpurun_out/r03s_pytest.log
timeout -k 10 400 python -u tools/nt_ab.py gpurun_out/r03s_nt_ab.json > gpurun_out/r03s_nt_ab.log 2>&1 || { tail -20 gpurun_out/r03s_nt_ab.log; exit 1; }
cat gpurun_out/r03s_nt_ab.json
