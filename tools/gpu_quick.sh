set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/me_variants.py > gpurun_out/me_variants.log 2>&1
echo "variants exit: $?" >> gpurun_out/me_variants.log
timeout -k 10 900 python -m pytest tests/test_gpu_me.py -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit: $?" >> gpurun_out/pytest_gpu.log
