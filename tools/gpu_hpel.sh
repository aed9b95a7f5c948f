# hpel_filter round: parity of every hpel variant, then the A/B timing at 16 and 64 frames
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mc.py -x -v -k hpel --timeout 120 --timeout-method thread > gpurun_out/pytest_hpel.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/hpel_variants.py 16 > gpurun_out/hpel_variants16.json 2>gpurun_out/hpel_variants16.err || exit 2
timeout -k 10 200 python -u tools/hpel_variants.py 64 > gpurun_out/hpel_variants64.json 2>gpurun_out/hpel_variants64.err || exit 3
echo done
