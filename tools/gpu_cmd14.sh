set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_ecfft.py tests/test_gpu_g2.py -x -q -m gpu > gpurun_out/pytest_ecfft.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ecfft.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/ecfft_bench.py bls12_381 10 12 14 16 18 > gpurun_out/ecfft.log 2>&1; echo "ecfft rc=$?"; cat gpurun_out/ecfft.log
