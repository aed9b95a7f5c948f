# bench + rocprofv3 kernel-trace/stats + two PMC passes (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
# the bench's own default command under the tracer (same warmup / steps as bench.log)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trace -o run -- python3 $R/bench.py > $R/gpurun_out/prof_trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/prof_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/prof_write.log 2>&1 || exit 4
echo done
