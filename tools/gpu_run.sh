# One parameterised GPU-box runner (replaces the per-session gpu_r03*.sh scripts).
# usage: bash tools/gpu_run.sh TAG STEP [STEP ...]
#   tests         full `-m gpu` suite            -> gpurun_out/TAG_pytest_gpu.log
#   tests:FILES   the named test files only (comma separated, under tests/)
#   smoke         __graft_entry__.smoke()        -> gpurun_out/TAG_smoke.log
#   bench         default bench.py               -> gpurun_out/TAG_bench.log
#   driver        bench.py --steps 20 --warmup 5 -> gpurun_out/TAG_bench_driver.log
#   profile       tools/gpu_profile.sh (trace + FETCH / WRITE PMC of the default bench)
#   py:SCRIPT     python tools/SCRIPT (args after '='), stdout -> gpurun_out/TAG_SCRIPT.log
#   envab:VAR     headline-only bench, VAR=0 / VAR=1 interleaved 3 times -> gpurun_out/TAG_envab.log
# Every GPU step runs under its own time limit; the first failing step ends the run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; shift
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 6; }
      tail -2 gpurun_out/${TAG}_pytest_gpu.log ;;
    tests:*)
      files=$(echo "${step#tests:}" | tr ',' '\n' | sed 's#^#tests/#' | tr '\n' ' ')
      timeout -k 10 600 python -u -m pytest $files -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 6; }
      tail -2 gpurun_out/${TAG}_pytest.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_smoke.log; exit 7; }
      cat gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 5; }
      tail -c 600 gpurun_out/${TAG}_bench.log; echo ;;
    driver)
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_bench_driver.log; exit 5; }
      tail -c 600 gpurun_out/${TAG}_bench_driver.log; echo ;;
    profile)
      rocm-smi --showclocks --showpower --showuse > gpurun_out/${TAG}_rocm_smi.txt 2>&1 || true
      bash tools/gpu_profile.sh || exit 8 ;;
    py:*)
      spec=${step#py:}; script=${spec%%=*}; args=""
      [ "$spec" != "$script" ] && args=$(echo "${spec#*=}" | tr ',' ' ')
      timeout -k 10 600 python -u tools/$script $args > gpurun_out/${TAG}_${script%.py}.log 2>&1 \
        || { tail -30 gpurun_out/${TAG}_${script%.py}.log; exit 9; }
      tail -30 gpurun_out/${TAG}_${script%.py}.log ;;
    envab:*)
      var=${step#envab:}
      for i in 1 2 3; do
        for v in 0 1; do
          env $var=$v timeout -k 10 200 python bench.py --no-cpu --no-extra > gpurun_out/${TAG}_ab.json 2>&1 \
            || { tail -20 gpurun_out/${TAG}_ab.json; exit 10; }
          echo "$var=$v $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/${TAG}_ab.json)" \
            | tee -a gpurun_out/${TAG}_envab.log
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
