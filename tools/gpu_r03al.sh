# round 3 (session 2): nontemporal 8/16-byte row stores in the fused reconstruction kernels: parity + A/B at 64 frames
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inverse.py > gpurun_out/r03al_pytest.log 2>&1 || { tail -30 gpurun_out/r03al_pytest.log; exit 1; }
tail -2 gpurun_out/r03al_pytest.log
timeout -k 10 300 python -u tools/recon_variants.py 64 gpurun_out/r03al_recon64.json > gpurun_out/r03al_recon64.log 2>&1 || { tail -20 gpurun_out/r03al_recon64.log; exit 2; }
cat gpurun_out/r03al_recon64.json
