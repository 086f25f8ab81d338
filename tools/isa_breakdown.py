"""Instruction-class breakdown of the NTT pass kernel's blocks (dev tool):
reads the device assembly tools/isa_count.py leaves in /tmp/isa_count.s and
sorts every instruction of the named kernel's blocks into the classes the
pass's cost model uses: product mads, 64-bit column shifts, Montgomery digits,
limb masks, limb-wise sums, LDS, address arithmetic, global memory, control.
Usage: python tools/isa_breakdown.py <symbol regex> [asm file]"""
import collections
import re
import sys

CLASSES = [
    ("mad (v_mad_u64_u32)", lambda op: op == "v_mad_u64_u32"),
    ("64-bit column shift", lambda op: op in ("v_lshrrev_b64", "v_ashrrev_i64", "v_lshlrev_b64")),
    ("Montgomery digit", lambda op: op in ("v_bitop3_b32", "v_mul_lo_u32")),
    ("limb mask", lambda op: op.startswith("v_and_b32") or op.startswith("v_and_or_b32")),
    ("limb sums", lambda op: op.startswith(("v_add_u32", "v_sub_u32", "v_add3_u32", "v_subrev_u32",
                                             "v_add_co", "v_addc", "v_sub_co", "v_subb", "v_lshl_add_u64",
                                             "v_mad_i64_i32"))),
    ("LDS", lambda op: op.startswith("ds_")),
    ("global memory", lambda op: op.startswith(("global_", "buffer_"))),
    ("address / other VALU", lambda op: op.startswith("v_")),
    ("wait / nop / scalar / branch", lambda op: True),
]


def classify(op):
    for name, pred in CLASSES:
        if pred(op):
            return name


def main():
    pat = re.compile(sys.argv[1])
    path = sys.argv[2] if len(sys.argv) > 2 else "/tmp/isa_count.s"
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat.search(l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name, loop = [], collections.Counter(), "entry", False
    for l in lines[start + 1:end]:
        if re.match(r"^\.LBB\S*:|^; %bb\.", l):
            blocks.append((name, loop, cur))
            name, loop, cur = l.split()[0].rstrip(":") if l.startswith(".") else l.split()[1], "Loop" in l, \
                collections.Counter()
            continue
        t = l.split()
        if not t or t[0].startswith((";", ".")):
            continue
        cur[classify(t[0])] += 1
    blocks.append((name, loop, cur))
    print(lines[start].split(":")[0][:120])
    hdr = "".join(f"{n.split(' ')[0][:9]:>10s}" for n, _ in CLASSES)
    print(f"{'block':14s}{'':2s}{hdr}{'VALU':>8s}")
    for name, loop, c in blocks:
        tot = sum(c.values())
        if tot < 40:
            continue
        valu = sum(v for k, v in c.items() if k not in ("LDS", "global memory", "wait / nop / scalar / branch"))
        print(f"{name:14s}{'L ' if loop else '  '}" + "".join(f"{c[n]:10d}" for n, _ in CLASSES) + f"{valu:8d}")
    print("classes:", ", ".join(n for n, _ in CLASSES))


if __name__ == "__main__":
    main()
