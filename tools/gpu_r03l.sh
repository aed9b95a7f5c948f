# headline batch size under the driver's arguments: 64 vs 128 pairs per step, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do
  for F in 64 128; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu --frames $F > gpurun_out/r03l_bench_F${F}_$i.log 2>&1 || exit 1
  done
done
echo done
