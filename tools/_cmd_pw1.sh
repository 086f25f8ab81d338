set -o pipefail
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_pw1.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pw1.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python3 tools/msm_sizes.py 20 21 22 23 26 > gpurun_out/sizes_pw1.log 2>&1 && cat gpurun_out/sizes_pw1.log &&
ECG_MSM_PW1=0 timeout -k 10 300 python3 tools/msm_sizes.py 20 21 22 > gpurun_out/sizes_pw0.log 2>&1 && cat gpurun_out/sizes_pw0.log
