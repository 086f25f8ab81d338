# Round evidence in one call: GPU parity suite + smoke + default bench, the
# BN254 bench line, then rocprofv3 kernel-trace stats and the PMC passes.
set -o pipefail
TAG=${1:-r01f}
bash tools/gpu_full.sh || exit $?
timeout -k 10 600 python3 bench.py --curve bn254 --no-e2e --no-aux > gpurun_out/bench_bn254.log 2>&1; rc=$?; echo "bn254 bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh $TAG
