# SQ issue / stall counters of the lookahead kernels over tools/leg_time.py la (the P, slice, batch and B legs)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/pmc_la1 -o run -- python3 $R/tools/leg_time.py la 5 > $R/gpurun_out/pmc_la1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/pmc_la2 -o run -- python3 $R/tools/leg_time.py la 5 > $R/gpurun_out/pmc_la2.log 2>&1 || exit 2
echo done
