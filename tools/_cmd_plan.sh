set -o pipefail
bash tools/gpu.sh tests || exit 1
timeout -k 10 300 python3 tools/msm_sizes.py 20 22 23 23 24 > gpurun_out/sizes_plan16.log 2>&1 && cut -c1-110 gpurun_out/sizes_plan16.log &&
bash tools/gpu.sh bench
