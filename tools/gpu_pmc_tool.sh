# PMC passes over a tool script (first argument, e.g. tools/tesa_time.py): SQ issue/stall,
# cache and address path, HBM; one counter group per rocprofv3 run
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/pmc_t1 -o run -- python3 $R/$T > $R/gpurun_out/pmc_t1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum --output-format csv -d $R/gpurun_out/pmc_t2 -o run -- python3 $R/$T > $R/gpurun_out/pmc_t2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_t3 -o run -- python3 $R/$T > $R/gpurun_out/pmc_t3.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_t4 -o run -- python3 $R/$T > $R/gpurun_out/pmc_t4.log 2>&1 || exit 4
echo done
