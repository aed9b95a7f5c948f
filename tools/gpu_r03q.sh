# round 3 profile of the final headline: default bench, kernel trace + stats, FETCH / WRITE PMC
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
rocm-smi --showclocks --showpower --showuse > gpurun_out/rocm_smi.txt 2>&1 || true
bash tools/gpu_profile.sh || exit 1
echo done
