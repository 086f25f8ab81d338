set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread -k "boundary_form or grid_failure or prepared or grid_part or dist_grid_host or large_matches or 2p29 or 2p25" > gpurun_out/pytest_sel.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo bench rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --gpus 4 --transport host --single-device --no-cpu-baseline > gpurun_out/rehearsal_4_selflaunch.log 2>&1; echo rehearsal rc=$?
