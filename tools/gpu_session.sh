set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -E "gfx950|Marketing" | head -4 > gpurun_out/rocminfo.txt || true
nproc > gpurun_out/nproc.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/nproc.txt
timeout -k 10 120 ./tools/sad_peak > gpurun_out/sad_peak.txt 2>&1 && timeout -k 10 120 ./tools/qsad_probe > gpurun_out/qsad_probe.txt 2>&1 &&
timeout -k 10 400 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
echo "exit: $?"
