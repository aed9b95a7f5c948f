# PMC passes over tools/subpel_variants.py (qpel candidate kernels): SQ issue/stall, cache, HBM
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM --output-format csv -d $R/gpurun_out/pmc_sp1 -o run -- python3 $R/tools/subpel_variants.py > $R/gpurun_out/pmc_sp1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum --output-format csv -d $R/gpurun_out/pmc_sp2 -o run -- python3 $R/tools/subpel_variants.py > $R/gpurun_out/pmc_sp2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_sp3 -o run -- python3 $R/tools/subpel_variants.py > $R/gpurun_out/pmc_sp3.log 2>&1 || exit 3
echo done
