# rocprofv3 evidence for one tool command (e.g. "tools/leg_time.py esa 10"): kernel trace +
# stats, then SQ issue / stall, address path and HBM counter passes, one group per run
# usage: bash tools/gpu_leg_prof.sh TAG "tools/leg_time.py esa 10"
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; T=$2
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 $R/$T > $R/gpurun_out/${TAG}_trace.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/${TAG}_pmc1 -o run -- python3 $R/$T > $R/gpurun_out/${TAG}_pmc1.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/${TAG}_pmc2 -o run -- python3 $R/$T > $R/gpurun_out/${TAG}_pmc2.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_pmc3 -o run -- python3 $R/$T > $R/gpurun_out/${TAG}_pmc3.log 2>&1 || exit 4
echo done
