"""The Rust drop-in's MSM call (ecg_msm_ex, arkworks Affine records, base
cache) at 2^N on one GPU (dev tool): one cold call (upload + device
conversion + prepare + MSM), then cached calls (exponents only).  Run it under
different ECG_MSM_H2D_PASSES to A/B the exponent pipelining depth.
Usage: python tools/e2e_cached_ab.py [log_n] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

ln = int(sys.argv[1]) if len(sys.argv) > 1 else 26
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << ln
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(7)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**62 - 1)
d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 12345, 678910, n)
ark = np.zeros((n, 13), dtype=np.uint64)
ark[:, :12] = d_b.read(shape=(n, 12))
d_b.free()
kern = ecgpu.MultiexpKernel.create([prog], [], "bls12_381")
t = time.perf_counter()
r0 = kern.multiexp_ex(ark, E, 0, ark_affine=True, cache_bases=True)
cold = time.perf_counter() - t
warm = []
for _ in range(reps):
    t = time.perf_counter()
    r1 = kern.multiexp_ex(ark, E, 0, ark_affine=True, cache_bases=True)
    warm.append(time.perf_counter() - t)
print(json.dumps({"log_n": ln, "passes_env": os.environ.get("ECG_MSM_H2D_PASSES", "default"),
                  "cold_ms": cold * 1e3, "cached_ms": [w * 1e3 for w in warm], "equal": bool((r0 == r1).all())}),
      flush=True)
