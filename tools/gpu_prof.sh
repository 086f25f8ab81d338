# rocprofv3 evidence for profiles/: kernel-trace stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -o pipefail
R=$PWD
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-aux > $R/gpurun_out/prof_${TAG}_bench.log 2>&1 && echo trace-ok &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-aux --steps 1 --warmup 0 > $R/gpurun_out/pmc_fetch_${TAG}.log 2>&1 && echo fetch-ok &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-aux --steps 1 --warmup 0 > $R/gpurun_out/pmc_write_${TAG}.log 2>&1 && echo write-ok
