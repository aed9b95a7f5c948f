# round 3 (session 2): DCT+quant 4x4 one-wave workgroups for the packed 8x8 (variant 10): parity, A/B, PMC of the default
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dct.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ah_pytest.log 2>&1 || { tail -30 gpurun_out/r03ah_pytest.log; exit 1; }
tail -2 gpurun_out/r03ah_pytest.log
timeout -k 10 300 python tools/dq_time.py > gpurun_out/r03ah_dq_ab.log 2>&1 || { tail gpurun_out/r03ah_dq_ab.log; exit 2; }
cat gpurun_out/r03ah_dq_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r03ah_fetch -o run -- python3 $R/tools/dq_time.py 64 10 default > $R/gpurun_out/r03ah_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r03ah_write -o run -- python3 $R/tools/dq_time.py 64 10 default > $R/gpurun_out/r03ah_write.log 2>&1 || exit 4
cd $R && python3 tools/pmc_by_kernel.py mb_dct $(find gpurun_out/r03ah_fetch gpurun_out/r03ah_write -name '*counter_collection.csv') > gpurun_out/r03ah_pmc.txt && cat gpurun_out/r03ah_pmc.txt
