# A/B of two builds: x264-i386pic_amd/libx264hip_base.so (HEAD) vs libx264hip.so (working
# tree), headline bench legs alternated three times each on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  X264HIP_LIBRARY=$PWD/x264-i386pic_amd/libx264hip_base.so timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab_base_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab_new_$i.log 2>&1 || exit 2
done
echo done
