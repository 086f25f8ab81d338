# SQ counters for the MSM kernels, one pass per library / env config (dev tool).
# usage: bash tools/gpu_sq_ab.sh <log_n> <tag>=<lib>[,ENV=V] ...
set -o pipefail
R=$PWD; LOGN=$1; shift
mkdir -p $R/gpurun_out
for spec in "$@"; do
  tag=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*,}
  ( cd /tmp && export TMPDIR=/tmp && export ECGPU_LIB=$R/$lib && [ -n "$envs" ] && export $envs
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --kernel-trace -d $R/gpurun_out/sq_$tag -o run --output-format csv -- python3 $R/tools/msm_once.py $LOGN 1 > $R/gpurun_out/sq_$tag.log 2>&1 ) || { echo "sq $tag failed"; exit 1; }
  echo "== $tag"; python3 $R/tools/sq_summary.py $R/gpurun_out/sq_$tag/run_counter_collection.csv
done
