# round-2 check: smoke, the whole GPU parity suite (verbose, per-test timeout), default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
lscpu | grep -E "Model name|^CPU\(s\)" > gpurun_out/cpu.txt
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "exit: $rc"; exit $rc
