# round 3 (session 2): TESA scan occupancy A/B (1- / 2-row staging chunks at 5 waves per SIMD vs 4-row chunks at 4), parity of each build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in ck1w5 ck2w5; do
  X264HIP_LIBRARY=tools/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_tesa.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03as_pytest_$v.log 2>&1 || { tail -20 gpurun_out/r03as_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r03as_pytest_$v.log
done
for i in 1 2 3; do
  for v in base ck1w5 ck2w5; do
    TESA_LIB=tools/ab/lib_$v.so timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03as_${v}_$i.log 2>&1 || exit 2
    echo "$v $(grep -o '"tesa_launch_ms": [0-9.]*' gpurun_out/r03as_${v}_$i.log)"
  done
done
