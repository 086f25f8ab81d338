# window-padded per-block sorts: parity, then A/B against the global sort
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_msm_prep.py tests/test_gpu_g2.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pw.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/msm_ab.py 26 ECG_MSM_PW=0 ECG_MSM_PW=1 ECG_MSM_PW=1,ECG_MSM_SORTCFG=1
