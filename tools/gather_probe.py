"""Is the MSM accumulation waiting on its base gathers? (dev tool)
Times msm_accumulate (HIP events, ecg_last_kernel_time) at 2^N over prepared
bases that are all distinct (every gather misses L2 / MALL) against the same
number of terms over a 2^k-base set tiled (the gathers hit the caches).  Same
scalars, same plan, same instruction stream; only the gather locality differs.
Usage: python tools/gather_probe.py curve log_n [log_small]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

curve, log_n = sys.argv[1], int(sys.argv[2])
log_small = int(sys.argv[3]) if len(sys.argv) > 3 else 12
n = 1 << log_n
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(7)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**61 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
cid = ecgpu.CURVE_NAMES[curve]
lq = ecgpu.CURVE_FQ_LIMBS[cid]
res = {"curve": curve, "log_n": log_n}
for kind in ("distinct", f"tiled_2^{log_small}"):
    if kind == "distinct":
        d_xy = ecgpu.gen_bases_dev(prog, curve, 12345, 678910, n)
    else:
        small = ecgpu.gen_bases_dev(prog, curve, 12345, 678910, 1 << log_small).read(shape=(1 << log_small, 2 * lq))
        d_xy = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(np.tile(small, (n >> log_small, 1))))
    d_b = ecgpu.prepare_bases(prog, curve, d_xy, n)
    d_xy.free()
    ecgpu.msm_dev(prog, curve, d_b, d_e, n)
    best = 1e9
    for _ in range(3):
        ecgpu.msm_dev(prog, curve, d_b, d_e, n)
        ms, cnt = prog.kernel_time("msm_accumulate")
        best = min(best, ms / max(cnt, 1))
    res[kind + "_acc_ms"] = round(best, 3)
    d_b.free()
print(json.dumps(res), flush=True)
