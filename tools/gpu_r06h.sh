# round-6 GPU batch h: clock + instruction counters of the single 2^26 MSM vs one N = 8 grid share vs a range shard
set -o pipefail
R=$PWD; mkdir -p gpurun_out
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD \
   --kernel-trace --output-format csv -d $R/gpurun_out/pmc_gridclk -o run -- python3 $R/tools/grid_trace.py 26 bls12_381 3 \
   > $R/gpurun_out/pmc_gridclk.log 2>&1 ) || { echo "pmc failed"; tail -5 gpurun_out/pmc_gridclk.log; exit 1; }
python3 - <<'PY'
import csv, collections, re
rows = list(csv.DictReader(open("gpurun_out/pmc_gridclk/run_counter_collection.csv")))
tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open("gpurun_out/pmc_gridclk/run_kernel_trace.csv"))}
acc = collections.defaultdict(dict)
for r in rows:
    if "msm_accumulate" not in r["Kernel_Name"]: continue
    acc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
for d, c in sorted(acc.items(), key=lambda kv: int(kv[0])):
    t = tr.get(d)
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6 if t else float("nan")
    clk = c.get("GRBM_GUI_ACTIVE", 0) / (dur * 1e3) if dur == dur and dur > 0 else 0
    print(f"dispatch {d}: {dur:8.3f} ms  GRBM_GUI_ACTIVE/t = {clk:6.3f} GHz  " +
          "  ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
PY
