"""Window-size sweep of one prepared-bases MSM (dev tool): times the MSM
through ecg_multiple_multiexp with one line and one chunk, which accepts a
pinned window, against the planner's own choice (window_bits = 0).
Usage: python tools/c_sweep.py <log_n> <c> [<c> ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

ln, cs = int(sys.argv[1]), [int(x) for x in sys.argv[2:]]
n = 1 << ln
prog = ecgpu.program(ecgpu.Device(0))
E = np.random.default_rng(7).integers(0, 2**64, size=(n, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**62 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 12345, 678910, n)
pb = ecgpu.prepare_bases(prog, "bls12_381", d_b, n)
d_b.free()
ref = None
for c in [0] + cs:
    run = lambda: ecgpu.multiple_multiexp(prog, pb, (d_e, n), 1, window_size=c, pin_window=c != 0)  # noqa: E731
    out = run()
    ref = out if ref is None else ref
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        run()
        best = min(best, time.perf_counter() - t)
    print(json.dumps({"log_n": ln, "c": c or "plan", "ms": best * 1e3, "same": bool((out == ref).all())}), flush=True)
