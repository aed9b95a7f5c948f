# PMC diagnostics of the full-search kernel: clock (GRBM_GUI_ACTIVE) and SQ issue/stall counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/pmc_sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
echo done
