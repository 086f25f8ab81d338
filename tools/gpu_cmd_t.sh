set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_msm.py -x -q -k "ragged" --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_t.log; exit $rc
