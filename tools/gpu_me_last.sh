# last-column kernel: ME parity (1080p / 4K / golden), then the two-build bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_me.py tests/test_gpu_4k.py tests/test_gpu_golden.py tests/test_gpu_tesa.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_me_last.log 2>&1 || exit 1
bash tools/gpu_ab.sh || exit 2
echo done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_last -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-extra --steps 30 --warmup 60 > $GRAFT_REPO_ROOT/gpurun_out/prof_last.log 2>&1 || exit 3
echo done2
