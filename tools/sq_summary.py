"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (dev tool).

Prints, per kernel (largest SQ_WAVE_CYCLES / dispatch count first), every
counter summed over dispatches, per wave, and the VALU mix: INT64 (the
v_mad_u64_u32 products), INT32 and other VALU instructions."""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for row in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"<.*", "", re.sub(r"\(.*$", "", row["Kernel_Name"]).replace("void ", ""))
    acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
    disp[name].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
order = sorted(acc.items(), key=lambda kv: -(kv[1].get("SQ_WAVE_CYCLES", 0) or kv[1].get("SQ_INSTS_VALU", 0)))
for name, c in order[:8]:
    waves = c.get("SQ_WAVES", 0) or 1
    print(f"== {name[:60]}  dispatches={len(disp[name])}")
    for k, v in sorted(c.items()):
        print(f"   {k:26s} {v:.4e}  per-wave {v / waves:.4e}")
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_VALU_INT64" in c:
        v = c["SQ_INSTS_VALU"]
        i64 = c["SQ_INSTS_VALU_INT64"]
        i32 = c.get("SQ_INSTS_VALU_INT32", 0)
        print(f"   VALU mix: int64 {i64 / v:.3f}  int32 {i32 / v:.3f}  other {(v - i64 - i32) / v:.3f}")
