set -o pipefail
R=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ecfft.py tests/test_gpu_g2.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ecfft.log 2>&1; rc=$?; echo pytest=$rc; tail -3 gpurun_out/pytest_ecfft.log
[ $rc -eq 0 ] || exit $rc
for W in 1 0; do
  ECG_ECFFT_WIN=$W timeout -k 10 300 python3 tools/ecfft_bench.py bls12_381 10 12 14 16 > gpurun_out/ecfft_win$W.log 2>&1 || exit 1
  ECG_ECFFT_WIN=$W timeout -k 10 300 python3 tools/ecfft_bench.py bn254 12 16 > gpurun_out/ecfft_bn_win$W.log 2>&1 || exit 1
  ECG_ECFFT_WIN=$W timeout -k 10 300 python3 tools/ecfft_g2_ab.py bls12_381_g2 10 12 > gpurun_out/ecfft_g2_win$W.log 2>&1 || exit 1
done
