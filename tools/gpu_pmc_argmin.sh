# counters of the ESA table argmin over tools/leg_time.py's esa leg (kernel-filtered)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
K="--kernel-include-regex me_esa_argmin"
timeout -s KILL 120 rocprofv3 $K --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_am1 -o run -- python3 $R/tools/leg_time.py esa 5 > $R/gpurun_out/pmc_am1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_am2 -o run -- python3 $R/tools/leg_time.py esa 5 > $R/gpurun_out/pmc_am2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 $K --pmc TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_am3 -o run -- python3 $R/tools/leg_time.py esa 5 > $R/gpurun_out/pmc_am3.log 2>&1 || exit 3
echo done
