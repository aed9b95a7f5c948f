# strip-height sweep of the default (variant 3) streaming hpel kernel at 16 and 64 frames
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/hpel_tune.py 16 > gpurun_out/hpel_rows16.json 2> gpurun_out/hpel_rows16.err || exit 1
timeout -k 10 200 python -u tools/hpel_tune.py 64 > gpurun_out/hpel_rows64.json 2> gpurun_out/hpel_rows64.err || exit 2
echo done
