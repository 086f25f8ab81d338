# reduction segment length with the merge tree (round 6)
set -o pipefail
R=$GRAFT_REPO_ROOT
for L in 20 23; do
  timeout -k 10 400 python3 tools/msm_ab.py $L ECG_MSM_RED_SEG=8 ECG_MSM_RED_SEG=4 ECG_MSM_RED_SEG=2 > $R/gpurun_out/tree_ls_$L.log 2>&1 || exit 1
  cat $R/gpurun_out/tree_ls_$L.log
done
AB_CURVE=bn254 timeout -k 10 300 python3 tools/msm_ab.py 20 ECG_MSM_RED_SEG=8 ECG_MSM_RED_SEG=4 > $R/gpurun_out/tree_ls_bn20.log 2>&1 && cat $R/gpurun_out/tree_ls_bn20.log
