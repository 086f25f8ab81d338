"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu.sh prof)
into profiles/<tag>/pmc_fetch_write.json (mean KB per dispatch per kernel) and
copy the kernel-trace stats next to it.  Usage: python tools/pmc_summary.py <tag>"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

tag = sys.argv[1]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = os.path.join(root, "profiles", tag)
os.makedirs(out_dir, exist_ok=True)
res = defaultdict(dict)
for ctr, sub in (("FETCH_SIZE", f"pmc_fetch_{tag}"), ("WRITE_SIZE", f"pmc_write_{tag}")):
    path = os.path.join(root, "gpurun_out", sub, "run_counter_collection.csv")
    acc = defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != ctr:
                continue
            name = re.sub(r"\(.*$", "", row["Kernel_Name"])          # drop the argument list
            name = re.sub(r"^void ", "", name)
            name = re.sub(r"<.*", "", name)                          # drop template args
            acc[name][0] += float(row["Counter_Value"])
            acc[name][1] += 1
    for name, (tot, cnt) in acc.items():
        res[name][ctr] = {"dispatches": cnt, "mean_kb": tot / cnt}
    shutil.copy(path, os.path.join(out_dir, f"pmc_{ctr.split('_')[0].lower()}_counters.csv"))
with open(os.path.join(out_dir, "pmc_fetch_write.json"), "w") as f:
    json.dump(res, f, indent=1, sort_keys=True)
# the copy bench.py reads on the GPU box (profiles/r*/ stays out of the gpurun push)
with open(os.path.join(root, "profiles", "pmc_current.json"), "w") as f:
    json.dump({"source": f"profiles/{tag}/pmc_fetch_write.json", "kernels": res}, f, indent=1, sort_keys=True)
stats = os.path.join(root, "gpurun_out", f"prof_{tag}", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(out_dir, "kernel_stats.csv"))
for k in ("msm_accumulate", "ntt_pass"):
    for n, v in res.items():
        if k in n:
            print(n, {c: round(x["mean_kb"] / 1e6, 3) for c, x in v.items()}, "GB (KB/1e6)")
