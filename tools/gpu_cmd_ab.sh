set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu -k "msm or batch or prep or dist" --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 tools/lib_ab.py "$@" > gpurun_out/lib_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/lib_ab.log
