set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ecfft_bench.py bls12_381 10 12 14 16 18 > gpurun_out/ecfft.log 2>&1; rc=$?; echo "ecfft rc=$rc"; cat gpurun_out/ecfft.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ecfft_bench.py bn254 12 16 > gpurun_out/ecfft_bn.log 2>&1; rc=$?; echo "ecfft bn rc=$rc"; cat gpurun_out/ecfft_bn.log
