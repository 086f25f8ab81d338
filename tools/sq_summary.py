"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (dev tool)."""
import csv, re, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"<.*", "", re.sub(r"\(.*$", "", row["Kernel_Name"]).replace("void ", ""))
    acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
for name, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:6]:
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{name[:40]:40s} valu_insts={c.get('SQ_INSTS_VALU', 0):.3e} active_valu/wave_cyc={c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} "
          f"wait_any/wave_cyc={c.get('SQ_WAIT_ANY', 0) / wc:.3f} wait_inst_any/wave_cyc={c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} "
          f"active_any/wave_cyc={c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} busy={c.get('SQ_BUSY_CYCLES', 0):.3e} wave_cyc={wc:.3e}")
