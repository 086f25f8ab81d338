set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_fft.py tests/test_gpu_dist.py -x -q -m gpu > gpurun_out/pytest_fft.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_fft.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/ntt_ab.py 24 ECG_NTT_FULLTW=0 ECG_NTT_FULLTW=1 ECG_NTT_FULLTW=1,ECG_NTT_MAXDEG=12 ECG_NTT_FULLTW=1,ECG_NTT_MAXDEG=8 > gpurun_out/ntt_ab.log 2>&1; echo "ntt_ab rc=$?"; cat gpurun_out/ntt_ab.log
