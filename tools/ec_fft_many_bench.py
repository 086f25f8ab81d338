"""radix_ec_fft_many over same-size, same-omega inputs (batched into one
transform per context) against the same inputs one radix_ec_fft call at a
time (dev tool).  Usage: python tools/ec_fft_many_bench.py [log_n] [count]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 14
count = int(sys.argv[2]) if len(sys.argv) > 2 else 8
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
P = int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab", 16)
w = pow(7, (R - 1) >> 32, R)
for _ in range(log_n, 32):
    w = w * w % R
x = w * (1 << 256) % R
om = np.array([(x >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
prog = ecgpu.program(ecgpu.Device(0))
k = ecgpu.EcFftKernel.create([prog], "bls12_381")
one = np.array([((1 << 384) % P >> (64 * i)) & (2**64 - 1) for i in range(6)], dtype=np.uint64)
n = 1 << log_n
ins = []
for c in range(count):
    pts = ecgpu.gen_bases_dev(prog, "bls12_381", 3 + c, 7, n).read(shape=(n, 12))
    ins.append(np.ascontiguousarray(np.concatenate([pts, np.tile(one, (n, 1))], axis=1)))
ref = [a.copy() for a in ins]
for a in ref:
    k.radix_ec_fft(a, om, log_n)
res = {}
for name in ("one_by_one", "many"):
    best = 1e9
    for _ in range(2):
        xs = [a.copy() for a in ins]
        t = time.perf_counter()
        if name == "many":
            k.radix_ec_fft_many(xs, [om] * count, [log_n] * count)
        else:
            for a in xs:
                k.radix_ec_fft(a, om, log_n)
        best = min(best, time.perf_counter() - t)
    res[name] = best * 1e3
    assert all((a == r).all() for a, r in zip(xs, ref)), name
print({"log_n": log_n, "count": count, "ms_one_by_one": round(res["one_by_one"], 2), "ms_many": round(res["many"], 2),
       "speedup": round(res["one_by_one"] / res["many"], 2)})
