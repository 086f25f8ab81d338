# EC-FFT butterflies in the reduced-radix form (+ 2-wave twin) and full-line base records: parity, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ecfft.py tests/test_gpu_g2.py tests/test_gpu_msm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ecfft.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ecfft.log; [ $rc -eq 0 ] || exit $rc
for cfg in "ECG_ECFFT_RR=0" "ECG_ECFFT_RR=0 ECG_ECFFT_W2=0" "ECG_ECFFT_RR=1 ECG_ECFFT_W2=0" "ECG_ECFFT_RR=1"; do
  echo "== $cfg"; env $cfg timeout -k 10 300 python3 tools/ecfft_bench.py bls12_381 14 16 2>&1 | grep -v "^CPU" | tail -3 || exit 1
done
timeout -k 10 800 python3 tools/lib_ab.py 0g-ec-gpu_amd/lib_old/libecgpu.so 0g-ec-gpu_amd/lib/libecgpu.so
