# round 3: profile of the tree with line-aligned hpel, nontemporal streaming stores, 8-row SSD
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 5
echo done
