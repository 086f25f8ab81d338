"""Time window-table MSMs (ecg_msm_prepare_table) against plain prepared bases
on one GPU (dev tool): prepare time, MSM time and the result check against
the plain-prepared MSM of the same inputs.
Usage: python tools/msm_table.py log_n c [c ...]   (c = 0: the engine's choice)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

ln, windows = int(sys.argv[1]), [int(x) for x in sys.argv[2:]] or [0]
curve = os.environ.get("CURVE", "bls12_381")
prog = ecgpu.program(ecgpu.Device(0))
n = 1 << ln
rng = np.random.default_rng(7)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**62 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
d_b = ecgpu.gen_bases_dev(prog, curve, 12345, 678910, n)


def timed(pb, reps=4):
    ecgpu.msm_dev(prog, curve, pb, d_e, n)
    best, acc = 1e9, 1e9
    for _ in range(reps):
        t = time.perf_counter()
        out = ecgpu.msm_dev(prog, curve, pb, d_e, n)
        best = min(best, time.perf_counter() - t)
        acc = min(acc, prog.kernel_time("msm_accumulate")[0])
    return out, best * 1e3, acc


pb = ecgpu.prepare_bases(prog, curve, d_b, n)
ref, ms, acc = timed(pb)
pb.free()
print(json.dumps({"log_n": ln, "form": "prepared", "ms": ms, "acc_ms": acc}), flush=True)
for c in windows:
    t = time.perf_counter()
    tab = ecgpu.prepare_bases(prog, curve, d_b, n, window_table=c)
    prep_s = time.perf_counter() - t
    out, ms, acc = timed(tab)
    tab.free()
    print(json.dumps({"log_n": ln, "form": "table", "c": c, "prepare_s": prep_s, "ms": ms, "acc_ms": acc,
                      "terms_per_s": n / ms * 1e3, "equal": bool((out == ref).all())}), flush=True)
