# One entry point for GPU-box work (run under gpurun from the repo root).
#   bash tools/gpu.sh tests [pytest args]     -m gpu parity suite (+ smoke)
#   bash tools/gpu.sh bench [bench args]      one bench.py line -> gpurun_out/bench.log
#   bash tools/gpu.sh prof TAG                rocprofv3 kernel stats + FETCH/WRITE PMC passes
#   bash tools/gpu.sh sq TAG LOGN [COUNTERS]  one SQ counter pass over tools/msm_once.py
#   bash tools/gpu.sh round TAG               tests + smoke + bench + bn254 bench + prof
# Every GPU step runs under its own timeout and the steps are chained, so the
# first failure ends the call.
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out
cmd=${1:-tests}; shift || true

tests() {
  timeout -k 10 1200 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "$@" \
    > $R/gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || return $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 $R/gpurun_out/smoke.log
  return $rc
}

bench() {
  timeout -k 10 600 python3 bench.py "$@" > $R/gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 $R/gpurun_out/bench.log | cut -c1-1500
  return $rc
}

prof() {
  local TAG=$1
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv \
      -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-aux --no-table > $R/gpurun_out/prof_${TAG}_bench.log 2>&1 &&
    echo trace-ok &&
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch_$TAG -o run \
      --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-aux --no-table --steps 1 --warmup 0 \
      > $R/gpurun_out/pmc_fetch_${TAG}.log 2>&1 && echo fetch-ok &&
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write_$TAG -o run \
      --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-aux --no-table --steps 1 --warmup 0 \
      > $R/gpurun_out/pmc_write_${TAG}.log 2>&1 && echo write-ok )
}

sq() {
  local TAG=$1 LOGN=$2
  local CTRS=${3:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"}
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace -d $R/gpurun_out/sq_$TAG -o run --output-format csv \
      -- python3 $R/tools/msm_once.py $LOGN 1 > $R/gpurun_out/sq_$TAG.log 2>&1 ) || { echo "sq $TAG failed"; return 1; }
  python3 $R/tools/sq_summary.py $R/gpurun_out/sq_$TAG/run_counter_collection.csv | tee $R/gpurun_out/sq_${TAG}_summary.txt
}

# one counter pass over any python target: pmc TAG "CTR ..." script.py args...
pmc() {
  local TAG=$1 CTRS=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace -d $R/gpurun_out/pmc_$TAG -o run --output-format csv \
      -- python3 "$@" > $R/gpurun_out/pmc_$TAG.log 2>&1 ) || { echo "pmc $TAG failed"; return 1; }
  echo "pmc $TAG ok"
}

# diagnostics: in-kernel clock (GRBM) + SQ instruction mix of the MSM accumulate
# (both curves) and of the NTT pass
diag() {
  local TAG=$1 SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
  local SQ2="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  pmc ${TAG}_clk_bls "GRBM_GUI_ACTIVE GRBM_COUNT" $R/tools/msm_once.py 26 16 1 bls12_381 &&
  pmc ${TAG}_clk_bn "GRBM_GUI_ACTIVE GRBM_COUNT" $R/tools/msm_once.py 26 20 1 bn254 &&
  pmc ${TAG}_sq_bls "$SQ1" $R/tools/msm_once.py 24 1 1 bls12_381 &&
  pmc ${TAG}_sq_bn "$SQ1" $R/tools/msm_once.py 24 1 1 bn254 &&
  pmc ${TAG}_clk_ntt "GRBM_GUI_ACTIVE GRBM_COUNT" $R/tools/ntt_once.py 24 1000 &&
  pmc ${TAG}_sq_ntt "$SQ1" $R/tools/ntt_once.py 24 3 &&
  pmc ${TAG}_sq2_ntt "$SQ2" $R/tools/ntt_once.py 24 3
}

# BN254 counter passes (bench line's BN254 roofline.traffic): accumulate at 2^26, NTT at 2^24
bnpmc() {
  local TAG=$1
  pmc ${TAG}_bn_acc_fetch "FETCH_SIZE" $R/tools/msm_once.py 26 1 1 bn254 &&
  pmc ${TAG}_bn_acc_write "WRITE_SIZE" $R/tools/msm_once.py 26 1 1 bn254 &&
  pmc ${TAG}_bn_ntt_fetch "FETCH_SIZE" $R/tools/ntt_once.py 24 3 bn254_fr &&
  pmc ${TAG}_bn_ntt_write "WRITE_SIZE" $R/tools/ntt_once.py 24 3 bn254_fr
}

case $cmd in
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  prof) prof "$@" ;;
  sq) sq "$@" ;;
  diag) diag "$@" ;;
  bnpmc) bnpmc "$@" ;;
  round)
    TAG=$1
    tests && bench && {
      timeout -k 10 600 python3 bench.py --curve bn254 --no-e2e > $R/gpurun_out/bench_bn254.log 2>&1; rc=$?
      echo "bn254 bench rc=$rc"; [ $rc -eq 0 ]; } && prof $TAG ;;
  *) echo "unknown subcommand $cmd"; exit 2 ;;
esac
