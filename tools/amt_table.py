"""Batched MSM on the AMT shape (ag-cuda-ec benches/amt.rs: 10 lines x 2^21,
1024 chunks per line) over plain prepared bases and over a window table (dev
tool; profile with rocprofv3 --kernel-trace --stats).
Usage: python tools/amt_table.py [window ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

windows = [int(x) for x in sys.argv[1:]] or [12]
L, lines, chunks = 1 << 21, 10, 1 << 10
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(5)
E = rng.integers(0, 2**64, size=(L, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**60 - 1)
d_le = ecgpu.DeviceBuffer.upload(prog, E)
d_lb = ecgpu.gen_bases_dev(prog, "bls12_381", 7, 11, L * lines)


def timed(b):
    ecgpu.multiple_multiexp(prog, b, (d_le, L), chunks)
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        out = ecgpu.multiple_multiexp(prog, b, (d_le, L), chunks)
        best = min(best, time.perf_counter() - t)
    return out, best * 1e3


pb = ecgpu.prepare_bases(prog, "bls12_381", d_lb, L * lines)
ref, ms = timed(pb)
pb.free()
print(json.dumps({"form": "prepared", "ms": ms, "acc_ms": prog.kernel_time("msm_accumulate")[0]}), flush=True)
for c in windows:
    tab = ecgpu.prepare_bases(prog, "bls12_381", d_lb, L * lines, window_table=c)
    out, ms = timed(tab)
    tab.free()
    print(json.dumps({"form": "table", "c": c, "ms": ms, "acc_ms": prog.kernel_time("msm_accumulate")[0],
                      "equal": bool((out == ref).all())}), flush=True)
