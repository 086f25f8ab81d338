set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu -k "msm or smoke or batch or prep or dist" --timeout 300 --timeout-method thread > gpurun_out/pytest_rr.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_rr.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/msm_ab.py 26 ECG_MSM_RR=0 ECG_MSM_RR=1 > gpurun_out/msm_ab_rr.log 2>&1; echo "ab rc=$?"; cat gpurun_out/msm_ab_rr.log
