set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_me.py tests/test_gpu_me_bind.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03j_pytest.log 2>&1 || exit 1
echo done
