# round 3 call c: ME XCD-remap A/B (+ FETCH_SIZE per variant), the bench (driver args)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/me_xcd_ab.py gpurun_out/r03c_me_xcd.json > gpurun_out/r03c_me_xcd.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
X264HIP_ME_XCD=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r03c_fetch0 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-extra --frames 16 > $R/gpurun_out/r03c_fetch0.log 2>&1 || exit 2
X264HIP_ME_XCD=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r03c_fetch1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-extra --frames 16 > $R/gpurun_out/r03c_fetch1.log 2>&1 || exit 3
cd $R
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03c_bench_driver.log 2>&1 || exit 4
echo done
