# hpel parity + A/B timing, ME parity, then the two-build bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_me.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mc_me.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/hpel_variants.py 16 > gpurun_out/hpel_variants16.json 2>gpurun_out/hpel_variants16.err || exit 2
timeout -k 10 200 python -u tools/hpel_variants.py 64 > gpurun_out/hpel_variants64.json 2>gpurun_out/hpel_variants64.err || exit 3
bash tools/gpu_ab.sh || exit 4
echo done
