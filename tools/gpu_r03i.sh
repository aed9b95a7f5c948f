set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/stream_var_ab.py gpurun_out/r03i_stream_var.json > gpurun_out/r03i_stream_var.log 2>&1 || exit 1
echo done
