# round-6 GPU batch d: batch-affine vs XYZZ mixed-add cost microbenchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/batch_affine_bench.py > gpurun_out/batch_affine_bench.log 2>&1; rc=$?
cat gpurun_out/batch_affine_bench.log; exit $rc
