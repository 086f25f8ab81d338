set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r01b
