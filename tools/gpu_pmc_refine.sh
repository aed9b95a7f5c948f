# refine_subpel's LDS-window A/B under rocprofv3 (tools/leg_time.py refine): kernel trace, then
# the SQ LDS / VALU counters and the address-path counters, each X264HIP_REFINE_STAGE = 1 / 0
# usage: bash tools/gpu_pmc_refine.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for st in 1 0; do
  export X264HIP_REFINE_STAGE=$st
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_s${st}_trace -o run -- python3 $R/tools/leg_time.py refine 10 > $R/gpurun_out/${TAG}_s${st}_trace.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/${TAG}_s${st}_pmc1 -o run -- python3 $R/tools/leg_time.py refine 10 > $R/gpurun_out/${TAG}_s${st}_pmc1.log 2>&1 || exit 2
  timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/${TAG}_s${st}_pmc2 -o run -- python3 $R/tools/leg_time.py refine 10 > $R/gpurun_out/${TAG}_s${st}_pmc2.log 2>&1 || exit 3
done
echo done
