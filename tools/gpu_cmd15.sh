set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/msm_ab.py 26 ECG_MSM_SORT=0 ECG_MSM_SORT=1 > gpurun_out/msm_ab.log 2>&1; echo "msm_ab rc=$?"; cat gpurun_out/msm_ab.log
