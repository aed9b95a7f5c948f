# round 3: PMC of the streaming frame kernels (hpel variant 7, lowres NT) at 64 frames
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/r03u_p1 -o run -- python3 $R/tools/stream_kern.py > $R/gpurun_out/r03u_p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r03u_p2 -o run -- python3 $R/tools/stream_kern.py > $R/gpurun_out/r03u_p2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r03u_p3 -o run -- python3 $R/tools/stream_kern.py > $R/gpurun_out/r03u_p3.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/r03u_p4 -o run -- python3 $R/tools/stream_kern.py > $R/gpurun_out/r03u_p4.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03u_tr -o run -- python3 $R/tools/stream_kern.py > $R/gpurun_out/r03u_tr.log 2>&1 || exit 5
cd $R && python3 tools/pmc_by_kernel.py "" $(find gpurun_out/r03u_p* -name '*counter_collection.csv') > gpurun_out/r03u_pmc.txt
cat gpurun_out/r03u_pmc.txt
find gpurun_out/r03u_tr -name '*kernel_stats.csv' -exec cat {} \;
