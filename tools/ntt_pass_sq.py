"""Per-pass SQ counter summary of the NTT (dev tool): groups a rocprofv3 --pmc
counter CSV by the full ntt_pass_rr_kernel instantiation (first pass reads the
boundary layout, inner passes planes, last pass writes the boundary layout)
and prints per-dispatch means and the derived VALU-busy / wait fractions.
Usage: python tools/ntt_pass_sq.py run_counter_collection.csv [more.csv ...]"""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"]
        if "ntt_pass" not in k:
            continue
        m = re.search(r"ntt_pass\w*<([^>]*)>", k)
        name = m.group(1) if m else k
        acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[name].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
for name, c in sorted(acc.items()):
    nd = max(len(disp[name]), 1)
    print(f"== ntt_pass_rr_kernel<{name}>  dispatches={nd}")
    for k, v in sorted(c.items()):
        print(f"   {k:24s} per-dispatch {v / nd:.4e}")
    w = c.get("SQ_WAVE_CYCLES")
    if w and "SQ_INSTS_VALU" in c:
        # 4 cycles per wave64 VALU instruction on one SIMD: issue-cycle share of wave lifetime
        print(f"   VALU issue cycles / wave cycles {4 * c['SQ_INSTS_VALU'] / w:.3f}")
    if w and "SQ_WAIT_ANY" in c:
        print(f"   SQ_WAIT_ANY / wave cycles      {c['SQ_WAIT_ANY'] / w:.3f}")
    if w and "SQ_WAIT_INST_ANY" in c:
        print(f"   SQ_WAIT_INST_ANY / wave cycles {c['SQ_WAIT_INST_ANY'] / w:.3f}")
    if "GRBM_GUI_ACTIVE" in c and "GRBM_COUNT" in c:
        print(f"   GRBM_GUI_ACTIVE / GRBM_COUNT   {c['GRBM_GUI_ACTIVE'] / c['GRBM_COUNT']:.3f}")
    if "SQ_BUSY_CYCLES" in c and "SQ_INSTS_VALU_INT64" in c:
        print(f"   v_mad share of VALU            {c['SQ_INSTS_VALU_INT64'] / c['SQ_INSTS_VALU']:.3f}")
