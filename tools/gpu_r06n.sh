# one-task reduction segments of 4 with the merge tree (default) vs 8 (pinned)
set -o pipefail
R=$GRAFT_REPO_ROOT
for L in 20 23; do
  timeout -k 10 400 python3 tools/msm_ab.py $L ECG_MSM_RED_SEG=8 "" > $R/gpurun_out/tree_ls4_$L.log 2>&1 || exit 1
  cat $R/gpurun_out/tree_ls4_$L.log
done
AB_CURVE=bn254 timeout -k 10 300 python3 tools/msm_ab.py 20 ECG_MSM_RED_SEG=8 "" > $R/gpurun_out/tree_ls4_bn20.log 2>&1 && cat $R/gpurun_out/tree_ls4_bn20.log
