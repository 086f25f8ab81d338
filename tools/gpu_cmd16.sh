set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sort -o run --output-format csv -- python3 $R/tools/msm_once.py 26 3 > $R/gpurun_out/prof_sort.log 2>&1; echo "prof rc=$?"
cd $R; python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/prof_sort/run_kernel_stats.csv')))
for r in rows[:16]:
    print(r['Name'][:70].ljust(70), r['Calls'], round(float(r['AverageNs'])/1e6, 3), 'ms')
PY
