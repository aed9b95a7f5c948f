set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_inverse.py -x -q > gpurun_out/pytest_inv.log 2>&1
rc=$?; echo "pytest exit: $rc" >> gpurun_out/pytest_inv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/recon_variants.py 16 > gpurun_out/recon16.log 2>&1
