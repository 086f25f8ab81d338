"""Effective clock of the heavy kernels from a GRBM_GUI_ACTIVE pass (dev tool):
clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md, DVFS)."""
import csv, os, re, sys
from collections import defaultdict
d = sys.argv[1]
dur = {}
for row in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    dur[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
acc = defaultdict(lambda: [0.0, 0.0, 0])
for row in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    if row["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    name = re.sub(r"<.*", "", re.sub(r"\(.*$", "", row["Kernel_Name"]).replace("void ", ""))
    a = acc[name]
    a[0] += float(row["Counter_Value"])
    a[1] += dur.get(row["Dispatch_Id"], 0.0)
    a[2] += 1
for name, (gui, t, n) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:5]:
    print(f"{name[:40]:40s} calls={n} ms/call={t / n * 1e3:8.3f} eff_clock={gui / 8 / t / 1e9 if t else 0:.3f} GHz")
