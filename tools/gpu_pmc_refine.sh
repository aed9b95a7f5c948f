# refine_subpel's counters under rocprofv3 (tools/leg_time.py refine: refine16 with chroma ME,
# refine16_luma, refine8, the me_search_ref legs): VALU / LDS / wait counters, then the
# address-path counters.  usage: bash tools/gpu_pmc_refine.sh TAG [LEG] (LEG: a tools/leg_time.py
# leg, default refine)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
LEG=${2:-refine}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/${TAG}_pmc1 -o run -- python3 $R/tools/leg_time.py $LEG 5 > $R/gpurun_out/${TAG}_pmc1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/${TAG}_pmc2 -o run -- python3 $R/tools/leg_time.py $LEG 5 > $R/gpurun_out/${TAG}_pmc2.log 2>&1 || exit 2
echo done
