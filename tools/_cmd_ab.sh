set -o pipefail
for s in 4 8 16 32; do
  echo "COMB_SEG=$s"; ECG_MSM_COMB_SEG=$s timeout -k 10 300 python3 tools/msm_sizes.py 20 23 26 || exit 1
done > gpurun_out/ab_comb.log 2>&1
for s in 4 8 16 32; do
  echo "RED_SEG=$s"; ECG_MSM_RED_SEG=$s timeout -k 10 300 python3 tools/msm_sizes.py 20 || exit 1
done > gpurun_out/ab_red20.log 2>&1
for s in 16 28 48 64; do
  echo "RED_SEG=$s"; ECG_MSM_RED_SEG=$s timeout -k 10 300 python3 tools/msm_sizes.py 23 || exit 1
done > gpurun_out/ab_red23.log 2>&1
cat gpurun_out/ab_comb.log gpurun_out/ab_red20.log gpurun_out/ab_red23.log | cut -c1-90
