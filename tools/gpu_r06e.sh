# round-6 GPU batch e: kernel trace of one rank's grid share (N = 8) vs the single MSM and a range shard
set -o pipefail
R=$PWD; mkdir -p gpurun_out
for C in bls12_381 bn254; do
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gridtrace_$C -o run \
    -- python3 $R/tools/grid_trace.py 26 $C 3 > $R/gpurun_out/gridtrace_$C.log 2>&1 ) || { echo "trace $C failed"; exit 1; }
f=$(find gpurun_out/gridtrace_$C -name "run_kernel_trace.csv" | head -1)
python3 tools/trace_segments.py "$f" 3 50 > gpurun_out/grid_trace_segments_$C.txt; cat gpurun_out/grid_trace_segments_$C.txt
done
