# round 3 (session 2): TESA scan: per-row ADS bounds precomputed and broadcast, lane activity folded into ads: parity + A/B against the previous build (tools/ab)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tesa.py tests/test_gpu_4k.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aq_pytest.log 2>&1 || { tail -30 gpurun_out/r03aq_pytest.log; exit 1; }
tail -2 gpurun_out/r03aq_pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03aq_new_$i.log 2>&1 || exit 2
  TESA_LIB=tools/ab/libx264hip_base.so timeout -k 10 200 python tools/tesa_time.py > gpurun_out/r03aq_base_$i.log 2>&1 || exit 3
done
grep -h tesa_launch gpurun_out/r03aq_new_*.log gpurun_out/r03aq_base_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l[l.index('{'):]); print(round(d['tesa_launch_ms'], 4), round(d['tesa_centred_table_step_ms'], 4))"
