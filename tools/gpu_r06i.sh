# round-6 GPU batch i: accumulate time vs size for both curves (is BN254's per-instruction gap size-dependent?)
set -o pipefail
mkdir -p gpurun_out
for L in 22 24 25 26; do
  timeout -k 10 300 python3 -u tools/msm_ab.py $L "" >> gpurun_out/acc_scaling_bls.log 2>&1 || exit 1
  AB_CURVE=bn254 timeout -k 10 300 python3 -u tools/msm_ab.py $L "" >> gpurun_out/acc_scaling_bn.log 2>&1 || exit 1
  echo "log $L"; tail -1 gpurun_out/acc_scaling_bls.log; tail -1 gpurun_out/acc_scaling_bn.log
done
