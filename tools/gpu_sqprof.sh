# SQ counter pass (VALU / wait breakdown) for the NTT and MSM hot kernels.
set -o pipefail
R=$PWD; TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/pmc_sq_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --msm-log 22 > $R/gpurun_out/pmc_sq_${TAG}.log 2>&1 && echo sq-ok
