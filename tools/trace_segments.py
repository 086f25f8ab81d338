"""Split a rocprofv3 kernel trace at idle gaps > GAP ms and print, for the
last K segments, each kernel's summed time and launches (dev tool).
Usage: python tools/trace_segments.py run_kernel_trace.csv [K] [GAP_ms]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gap = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
segs, cur, prev_end = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev_end is not None and (s - prev_end) / 1e6 > gap:
        segs.append(cur)
        cur = []
    cur.append(r)
    prev_end = e if prev_end is None else max(prev_end, e)
segs.append(cur)
for seg in segs[-K:]:
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    agg = collections.OrderedDict()
    for r in seg:
        name = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "")
        name = re.sub(r"<.*", "", name)
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a = agg.setdefault(name, [0.0, 0])
        a[0] += d
        a[1] += 1
    busy = sum(a[0] for a in agg.values())
    print(f"--- segment: span {(t1 - t0) / 1e6:.2f} ms, kernel busy {busy:.2f} ms")
    for name, (ms, cnt) in agg.items():
        print(f"  {ms:9.3f} ms  x{cnt:<4d} {name[:70]}")
