set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/field_bench > gpurun_out/field_bench.log 2>&1; echo "fb rc=$?"; cat gpurun_out/field_bench.log
