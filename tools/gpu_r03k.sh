set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_lookahead.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03k_pytest.log 2>&1 || exit 1
echo done
