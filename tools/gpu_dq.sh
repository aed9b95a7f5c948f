set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dct.py -x -q > gpurun_out/pytest_dct.log 2>&1
rc=$?; echo "pytest exit: $rc" >> gpurun_out/pytest_dct.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/dq_variants.py 16 > gpurun_out/dq16.log 2>&1 || exit 3
timeout -k 10 300 python tools/dq_variants.py 64 > gpurun_out/dq64.log 2>&1
