"""The reference's multiexp bench shape (ag-cuda-ec/benches/multiexp.rs:15-62:
2^22 terms cycled with periods 99 / 73, 1024 tasks of 4096) run a few times
through ecg_multiple_multiexp (profiling target, dev tool).
Usage: python tools/refshape_once.py [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd"), os.path.join(ROOT, "oracle")]
import coracle as co  # noqa: E402  (input generation only)
import ecgpu  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
prog = ecgpu.program(ecgpu.Device(0))
n = 1 << 22
meta_b = co.gen_bases(0, 41, 43, 99)
d_b = ecgpu.upload_multiexp_bases(prog, np.ascontiguousarray(np.resize(meta_b, (n, meta_b.shape[1]))),
                                  curve="bls12_381")
E = np.random.default_rng(73).integers(0, 2**64, size=(73, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**62 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(np.resize(E, (n, 4))))
best = 1e9
for _ in range(reps):
    t = time.perf_counter()
    ecgpu.multiple_multiexp(prog, d_b, (d_e, n), 1024, 8, False, curve="bls12_381")
    best = min(best, time.perf_counter() - t)
print(f"reference bench shape: best {best * 1e3:.2f} ms of {reps}")
