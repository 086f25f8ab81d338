set -o pipefail
for s in 0 56 0 56; do
  echo "RED_SEG=$s"; ECG_MSM_RED_SEG=$s timeout -k 10 300 python3 tools/msm_sizes.py 23 || exit 1
done > gpurun_out/ab_red23b.log 2>&1
for s in 0 104 0 104; do
  echo "RED_SEG=$s"; ECG_MSM_RED_SEG=$s timeout -k 10 300 python3 tools/msm_sizes.py 26 || exit 1
done > gpurun_out/ab_red26.log 2>&1
cat gpurun_out/ab_red23b.log gpurun_out/ab_red26.log | cut -c1-100
timeout -k 10 600 python3 bench.py > gpurun_out/bench_aux.log 2>&1; echo bench rc=$?; tail -1 gpurun_out/bench_aux.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['aux']['msm_2p20'])"
