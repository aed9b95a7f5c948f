# round-end evidence in one call: runtime tests (upload entry) first, then smoke, the whole
# GPU parity suite, the default bench, and the rocprofv3 trace + FETCH/WRITE PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showclocks --showpower --showuse > gpurun_out/rocm_smi.txt 2>&1 || true
timeout -k 10 200 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_runtime.log 2>&1 || exit 1
bash tools/gpu_r02.sh || exit 2
bash tools/gpu_profile.sh || exit 3
echo done
