# merge-tree A/B (round 6): parity subset, a 2^20 timeline, then interleaved A/Bs
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_prepared.py tests/test_gpu_table.py > $R/gpurun_out/tree_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $R/gpurun_out/tree_pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr20t -o run -- python3 $R/tools/msm_once.py 20 4 1 > /dev/null 2>&1 ) && python3 tools/trace_last.py gpurun_out/tr20t/run_kernel_trace.csv > gpurun_out/tr20t.txt 2>&1 && tail -22 gpurun_out/tr20t.txt
for L in 20 23 26; do
  timeout -k 10 500 python3 tools/msm_ab.py $L ECG_MSM_BITS_TREE=0 ECG_MSM_BITS_TREE=1 ECG_MSM_BITS_TREE=1,ECG_MSM_TREE_LANES=1 > $R/gpurun_out/tree_ab_$L.log 2>&1 || exit 1
  cat $R/gpurun_out/tree_ab_$L.log
done
AB_CURVE=bn254 timeout -k 10 300 python3 tools/msm_ab.py 20 ECG_MSM_BITS_TREE=0 ECG_MSM_BITS_TREE=1 > $R/gpurun_out/tree_ab_bn20.log 2>&1 && cat $R/gpurun_out/tree_ab_bn20.log
