# fused ESA: parity of the ME suite on the working tree, then esa_time.py over three builds
# (base = libx264hip_base.so, pf = libx264hip_pf.so, new = libx264hip.so) x load lead 1 / 2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_me.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_me.log 2>&1 || exit 1
L=$PWD/x264-i386pic_amd
for i in 1 2; do
  for lead in 1 2; do
    for b in base pf new; do
      lib=$L/libx264hip_$b.so; [ $b = new ] && lib=$L/libx264hip.so
      echo "$b lead$lead $(X264HIP_ME_LEAD=$lead X264HIP_LIBRARY=$lib timeout -k 10 120 python tools/esa_time.py 2>/dev/null | tail -1)" >> gpurun_out/esa_ab.txt || exit 2
    done
  done
done
echo done
