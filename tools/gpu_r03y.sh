# round 3: SSD default (8 rows) parity; TESA PMC (issue / wait breakdown of the scan kernel)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ssd_plane.py > gpurun_out/r03y_pytest.log 2>&1 || { tail -30 gpurun_out/r03y_pytest.log; exit 1; }
tail -2 gpurun_out/r03y_pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/r03y_t1 -o run -- python3 $R/tools/tesa_time.py > $R/gpurun_out/r03y_t1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/r03y_t2 -o run -- python3 $R/tools/tesa_time.py > $R/gpurun_out/r03y_t2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r03y_t3 -o run -- python3 $R/tools/tesa_time.py > $R/gpurun_out/r03y_t3.log 2>&1 || exit 3
cd $R && python3 tools/pmc_by_kernel.py "tesa" $(find gpurun_out/r03y_t* -name '*counter_collection.csv') > gpurun_out/r03y_pmc.txt
cat gpurun_out/r03y_pmc.txt
