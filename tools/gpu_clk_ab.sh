# Effective clock per kernel (GRBM_GUI_ACTIVE / 8 XCDs / kernel time), one pass per config (dev tool).
# usage: bash tools/gpu_clk_ab.sh <log_n> <tag>=<lib>[,ENV=V] ...
set -o pipefail
R=$PWD; LOGN=$1; shift
mkdir -p $R/gpurun_out
for spec in "$@"; do
  tag=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*,}
  ( cd /tmp && export TMPDIR=/tmp && export ECGPU_LIB=$R/$lib && [ -n "$envs" ] && export $envs
    timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_$tag -o run --output-format csv -- python3 $R/tools/msm_once.py $LOGN 2 > $R/gpurun_out/clk_$tag.log 2>&1 ) || { echo "clk $tag failed"; exit 1; }
  echo "== $tag"; python3 $R/tools/clk_summary.py $R/gpurun_out/clk_$tag
done
