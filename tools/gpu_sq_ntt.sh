# SQ counter passes for the NTT pass kernel (VALU / wait / LDS breakdown)
set -o pipefail
R=$PWD; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/sq_ntt1 -o run --output-format csv -- python3 $R/tools/ntt_once.py 24 5 > $R/gpurun_out/sq_ntt1.log 2>&1 && echo sq1-ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_WAIT_INST_LDS --kernel-trace -d $R/gpurun_out/sq_ntt2 -o run --output-format csv -- python3 $R/tools/ntt_once.py 24 5 > $R/gpurun_out/sq_ntt2.log 2>&1 && echo sq2-ok &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/sq_ntt3 -o run --output-format csv -- python3 $R/tools/ntt_once.py 24 5 > $R/gpurun_out/sq_ntt3.log 2>&1 && echo sq3-ok
