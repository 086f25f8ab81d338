"""Per-dispatch clock and fill of one kernel from a rocprofv3 --pmc run with
GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES, SQ_WAVES, SQ_INSTS_VALU and --kernel-trace
(dev tool).  Usage: python tools/clk_report.py <pmc dir> <kernel substring>"""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0])))
tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]))}
acc = collections.defaultdict(dict)
for r in rows:
    if pat in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
for disp, c in sorted(acc.items(), key=lambda kv: int(kv[0])):
    t = tr[disp]
    ms = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6
    ghz = c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e6)  # GRBM_GUI_ACTIVE sums the 8 XCDs
    fill = c["SQ_WAVE_CYCLES"] * 4 / (ms * 1e-3 * ghz * 1e9)
    print(f"{pat} dispatch {disp}: {ms:8.3f} ms  clock {ghz:5.3f} GHz  resident waves {fill:6.0f}  "
          f"VALU per wave {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.4g}")
