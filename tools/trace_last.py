"""Print the kernels of the last MSM call in a rocprofv3 kernel trace with
durations and the idle gaps before them (dev tool).
Usage: python tools/trace_last.py run_kernel_trace.csv [first_kernel_substring]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "msm_digits"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
seg = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows[starts[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "")
    name = re.sub(r"<.*", "", name)
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev_end) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {name[:60]}")
    busy += e - s
    prev_end = max(prev_end, e)
print(f"span {(prev_end - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us")
