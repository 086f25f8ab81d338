set -o pipefail
R=$PWD
timeout -k 10 300 python3 tools/msm_sizes.py 20 21 22 23 24 26 > gpurun_out/msm_sizes.log 2>&1 && cat gpurun_out/msm_sizes.log &&
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof23 -o run --output-format csv -- python3 $R/tools/msm_once.py 23 5 1 > $R/gpurun_out/prof23.log 2>&1 ) && echo prof-ok
