"""Host-slice MSM (the reference API's path: bases and exps copied in on every
call) at 2^N for one ECG_MSM_H2D_PASSES setting (dev tool).
Usage: ECG_MSM_H2D_PASSES=k python tools/e2e_ab.py [log_n]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import ecgpu  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
n = 1 << log_n
prog = ecgpu.program(ecgpu.Device(0))
d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 3, 5, n)
B = d_b.read(shape=(n, 12))
E = bench.rand_scalars(np.random.default_rng(1), n, bench.R_BLS)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
ref = ecgpu.msm_dev(prog, "bls12_381", d_b, d_e, n)
t0 = time.perf_counter()
ecgpu.msm_dev(prog, "bls12_381", d_b, d_e, n)
resident = time.perf_counter() - t0
d_b.free()
d_e.free()
k = ecgpu.MultiexpKernel.create([prog], [], "bls12_381")
k.multiexp(ecgpu.Worker(), B, E, 0)
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    out = k.multiexp(ecgpu.Worker(), B, E, 0)
    ts.append(time.perf_counter() - t0)
print(json.dumps({"passes": os.environ.get("ECG_MSM_H2D_PASSES", "4"), "log_n": log_n,
                  "resident_ms": resident * 1e3, "e2e_ms": [t * 1e3 for t in ts],
                  "equal": bool((out == ref).all())}), flush=True)
