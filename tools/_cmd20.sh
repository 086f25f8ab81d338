set -o pipefail
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof20 -o run --output-format csv -- python3 $R/tools/msm_once.py 20 10 1 > $R/gpurun_out/prof20.log 2>&1 ) && echo prof20-ok &&
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof22 -o run --output-format csv -- python3 $R/tools/msm_once.py 22 5 1 > $R/gpurun_out/prof22.log 2>&1 ) && echo prof22-ok
