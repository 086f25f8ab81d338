set -o pipefail
bash tools/gpu.sh tests || exit 1
timeout -k 10 300 python3 tools/msm_sizes.py 16 18 20 21 22 23 24 26 > gpurun_out/sizes_ls8.log 2>&1 && cat gpurun_out/sizes_ls8.log | cut -c1-100 &&
( echo "RED_SEG=3 at 2^18, 4 at 2^20 (previous defaults)"; ECG_MSM_RED_SEG=3 timeout -k 10 300 python3 tools/msm_sizes.py 18 && ECG_MSM_RED_SEG=4 timeout -k 10 300 python3 tools/msm_sizes.py 20 ) > gpurun_out/sizes_ls_old.log 2>&1 && cat gpurun_out/sizes_ls_old.log | cut -c1-100 &&
bash tools/gpu.sh bench
