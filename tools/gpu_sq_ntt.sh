# SQ counter passes for the NTT pass kernels, reduced-radix (rr) and 32-bit-limb (std) A/B
set -o pipefail
R=$PWD; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  export ECG_NTT_RR=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $R/gpurun_out/sq_ntt_rr$v -o run --output-format csv -- python3 $R/tools/ntt_once.py 24 5 > $R/gpurun_out/sq_ntt_rr$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM --kernel-trace -d $R/gpurun_out/sq_ntt_rr${v}b -o run --output-format csv -- python3 $R/tools/ntt_once.py 24 5 > $R/gpurun_out/sq_ntt_rr${v}b.log 2>&1 || exit 1
  echo "== ECG_NTT_RR=$v"
  python3 $R/tools/sq_summary.py $R/gpurun_out/sq_ntt_rr$v/run_counter_collection.csv | grep -A14 "ntt_pass"
  python3 $R/tools/sq_summary.py $R/gpurun_out/sq_ntt_rr${v}b/run_counter_collection.csv | grep -A14 "ntt_pass"
done
