"""Kernel-trace target for the grid split (dev tool): after a warm-up, one
single-GPU 2^n MSM, rank `r` of 8's grid step, and range shard 0 of 8, each
separated by 100 ms of idle so tools/trace_segments.py can split the trace.
Usage: python tools/grid_trace.py [log_n] [curve] [rank]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
curve = sys.argv[2] if len(sys.argv) > 2 else "bls12_381"
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n = 1 << log_n
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(11)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**60 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
d_raw = ecgpu.gen_bases_dev(prog, curve, 12345, 678910, n)
prep = ecgpu.prepare_bases(prog, curve, d_raw, n)
d_raw.free()
m = n // 8
shard = prep.view(0, m)


class _Ptr:
    def __init__(self, buf, off):
        self.ptr = ctypes.c_void_p(buf.ptr.value + off)


steps = [lambda: ecgpu.msm_dev(prog, curve, prep, d_e, n),
         lambda: ecgpu.msm_grid_part(prog, curve, prep, d_e, n, rank, 8),
         lambda: ecgpu.msm_dev(prog, curve, shard, _Ptr(d_e, 0), m)]
for f in steps:  # warm-up (workspaces)
    f()
for f in steps:
    time.sleep(0.1)
    t0 = time.perf_counter()
    f()
    print(f"{(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
