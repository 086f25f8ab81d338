"""Static instruction counts of one kernel in a libecgpu translation unit (dev
tool): compiles the unit to gfx950 assembly (device only), extracts the first
kernel whose symbol matches the pattern and prints, per basic block, the
VALU / v_mad_u64_u32 / LDS / s_nop counts plus the kernel histogram.
Loop blocks are marked.  Used to compare code variants without a GPU: the
dominant kernels are VALU-issue-bound, so VALU instructions per iteration are
the cost model.
Usage: python tools/isa_count.py <csrc/unit.hip> <symbol regex> [-DFLAG ...]
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "0g-ec-gpu_amd")


def main():
    unit, pat, flags = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3:]
    out = os.environ.get("ISA_S", "/tmp/isa_count.s")
    if not os.environ.get("ISA_S"):
      subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                             "--offload-device-only", "-S", *flags, unit, "-o", out], cwd=PKG,
                            stderr=subprocess.DEVNULL)
    lines = open(out).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat.search(l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end + 1]
    print(body[0].split(":")[0][:160])
    hist = collections.Counter()
    blocks = []
    cur = {"name": "entry", "valu": 0, "mad": 0, "lds": 0, "nop": 0, "loop": False}
    for l in body[1:]:
        if re.match(r"^\.LBB\S*:|^; %bb\.", l):
            blocks.append(cur)
            cur = {"name": l.split()[0].rstrip(":") if l.startswith(".") else l.split()[1], "valu": 0, "mad": 0,
                   "lds": 0, "nop": 0, "loop": "Loop" in l}
            continue
        t = l.split()
        if not t or t[0].startswith((";", ".")):
            continue
        op = t[0]
        hist[op] += 1
        if op.startswith("v_"):
            cur["valu"] += 1
            cur["mad"] += op == "v_mad_u64_u32"
        elif op.startswith("ds_"):
            cur["lds"] += 1
        elif op == "s_nop":
            cur["nop"] += 1
    blocks.append(cur)
    for b in blocks:
        if b["valu"] or b["lds"]:
            print(f"  {b['name']:14s} {'L' if b['loop'] else ' '} valu {b['valu']:6d} mad {b['mad']:6d} "
                  f"lds {b['lds']:4d} nop {b['nop']:5d}")
    tot = {k: sum(b[k] for b in blocks) for k in ("valu", "mad", "lds", "nop")}
    loop = {k: sum(b[k] for b in blocks if b["loop"]) for k in ("valu", "mad", "lds", "nop")}
    print("kernel:", tot)
    print("loop blocks:", loop)
    print("top ops:", ", ".join(f"{k} {v}" for k, v in hist.most_common(16)))


if __name__ == "__main__":
    main()
