set -o pipefail
bash tools/gpu.sh tests || exit 1
timeout -k 10 300 python3 tools/msm_sizes.py 18 20 22 > gpurun_out/sizes_ls8b.log 2>&1 && cut -c1-100 gpurun_out/sizes_ls8b.log &&
timeout -k 10 300 python3 tools/c_sweep.py 20 14 15 16 17 18 > gpurun_out/c_sweep20.log 2>&1 && cat gpurun_out/c_sweep20.log &&
timeout -k 10 300 python3 tools/c_sweep.py 23 16 17 18 19 20 > gpurun_out/c_sweep23.log 2>&1 && cat gpurun_out/c_sweep23.log &&
timeout -k 10 400 python3 tools/c_sweep.py 26 19 20 21 > gpurun_out/c_sweep26.log 2>&1 && cat gpurun_out/c_sweep26.log
