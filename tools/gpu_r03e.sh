set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/stream_check.py > gpurun_out/r03e_stream_check.log 2>&1 || exit 1
PROBE_FRAMES=60 timeout -k 10 300 python tools/stream_probe.py gpurun_out/r03e_stream_probe.json > gpurun_out/r03e_stream_probe.log 2>&1 || exit 2
echo done
