# round 3 (session 2): fused DCT+quant at 64 frames -- time, kernel trace, FETCH / WRITE PMC
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python tools/dq_time.py > gpurun_out/r03ae_dq_time.log 2>&1 || { tail gpurun_out/r03ae_dq_time.log; exit 1; }
cat gpurun_out/r03ae_dq_time.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03ae_trace -o run -- python3 $R/tools/dq_time.py > $R/gpurun_out/r03ae_trace.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r03ae_fetch -o run -- python3 $R/tools/dq_time.py 64 10 > $R/gpurun_out/r03ae_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r03ae_write -o run -- python3 $R/tools/dq_time.py 64 10 > $R/gpurun_out/r03ae_write.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $R/gpurun_out/r03ae_l2 -o run -- python3 $R/tools/dq_time.py 64 10 > $R/gpurun_out/r03ae_l2.log 2>&1 || exit 5
cd $R && python3 tools/pmc_by_kernel.py mb_dct $(find gpurun_out/r03ae_fetch gpurun_out/r03ae_write gpurun_out/r03ae_l2 -name '*counter_collection.csv') > gpurun_out/r03ae_pmc.txt && cat gpurun_out/r03ae_pmc.txt
find gpurun_out/r03ae_trace -name '*kernel_stats.csv' -exec cat {} \; | head -12
