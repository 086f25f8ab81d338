# round-6 GPU batch j: accumulate clock / fill / VALU per wave, both curves, 2^24 and 2^26
set -o pipefail
R=$PWD; mkdir -p gpurun_out
for C in bls12_381 bn254; do for L in 24 26; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES \
     --kernel-trace --output-format csv -d $R/gpurun_out/pmc_clk_${C}_$L -o run -- python3 $R/tools/msm_once.py $L 2 1 $C \
     > $R/gpurun_out/pmc_clk_${C}_$L.log 2>&1 ) || { echo "pmc $C $L failed"; exit 1; }
  python3 tools/clk_report.py gpurun_out/pmc_clk_${C}_$L msm_accumulate | tee -a gpurun_out/acc_clock.txt
done; done
