# round-6 record, part 2: bench (BLS12-381, BN254), rocprof kernel stats + PMC passes, BN254 PMC passes
set -o pipefail
R=$PWD; mkdir -p gpurun_out
T=${1:-r06g}
bash tools/gpu.sh bench || exit 1
timeout -k 10 600 python3 -u bench.py --curve bn254 --no-e2e > gpurun_out/bench_bn254.log 2>&1; rc=$?
echo "bn254 bench rc=$rc"; tail -1 gpurun_out/bench_bn254.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/gpu.sh prof $T || exit 1
bash tools/gpu.sh bnpmc $T || exit 1
