# round 3: HBM pattern probe (store flavours, grid shapes) at 16 and 64 frames, then the
# streaming kernels' A/B with nontemporal stores
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./tools/stream_pattern 64 > gpurun_out/r03r_pattern64.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/stream_pattern 16 > gpurun_out/r03r_pattern16.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_var_ab.py gpurun_out/r03r_stream_nt.json > gpurun_out/r03r_stream_nt.log 2>&1 || exit 1
cat gpurun_out/r03r_pattern64.txt gpurun_out/r03r_pattern16.txt gpurun_out/r03r_stream_nt.json
