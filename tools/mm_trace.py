"""The reference's multiexp bench shape (ag-cuda-ec benches/multiexp.rs:15-62:
2^22 terms, bases cycled with period 99, scalars with period 73, 1024 tasks
of 4096) run K times on prepared bases, for a kernel trace (dev tool).
Usage: python tools/mm_trace.py [curve] [K] [table]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd"), os.path.join(ROOT, "oracle"), ROOT]
import ecgpu, coracle as co, bench
curve = sys.argv[1] if len(sys.argv) > 1 else "bls12_381"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
table = len(sys.argv) > 3 and sys.argv[3] == "table"
cid = ecgpu.CURVE_NAMES[curve]
lq = ecgpu.CURVE_FQ_LIMBS[cid]
r = bench.R_BLS if cid == 0 else bench.R_BN
prog = ecgpu.program(ecgpu.Device(0))
n = 1 << 22
hb = np.ascontiguousarray(np.resize(co.gen_bases(cid, 41, 43, 99), (n, 2 * lq)))
he = np.ascontiguousarray(np.resize(bench.rand_scalars(np.random.default_rng(73), 73, r), (n, 4)))
d_b = ecgpu.upload_multiexp_bases(prog, hb, curve=curve, window_table=0 if table else None)
d_e = ecgpu.DeviceBuffer.upload(prog, he)
ts = []
for _ in range(K + 1):
    t = time.perf_counter()
    o = ecgpu.multiple_multiexp(prog, d_b, (d_e, n), 1024, 8, False, curve=curve)
    ts.append(time.perf_counter() - t)
print(f"{curve} multiexp shape{' (table)' if table else ''}: best {min(ts[1:]) * 1e3:.2f} ms over {K}", flush=True)
