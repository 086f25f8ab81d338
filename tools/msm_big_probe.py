"""One large prepared G1 MSM against its known answer (dev tool): bases
(a + i b) G generated on the GPU and prepared, scalars uniform < r (seeded),
result vs (sum_i s_i (a + i b) mod r) G; timed twice (first call allocates).  Usage: python tools/msm_big_probe.py LOG_N [curve]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd"), os.path.join(ROOT, "oracle"), ROOT]
import ecgpu, coracle as co, bench
log_n = int(sys.argv[1]); curve = sys.argv[2] if len(sys.argv) > 2 else "bls12_381"
cid = ecgpu.CURVE_NAMES[curve]; n = 1 << log_n
r = bench.R_BLS if cid == 0 else bench.R_BN
prog = ecgpu.program(ecgpu.Device(0))
t = time.time()
scal = bench.rand_scalars(np.random.default_rng(log_n), n, r)
d_e = ecgpu.DeviceBuffer.upload(prog, scal)
raw = ecgpu.gen_bases_dev(prog, curve, 12345, 6789, n)
prep = ecgpu.prepare_bases(prog, curve, raw, n)
raw.free()
print(f"inputs ready {time.time() - t:.1f} s", flush=True)
# the first call grows the workspace (device allocations); the second runs on it
for call in ("first (allocates workspace)", "second (resident workspace)"):
    t = time.time()
    out = ecgpu.msm_dev(prog, curve, prep, d_e, n)
    print(f"msm {call}: {time.time() - t:.3f} s", flush=True)
k = co.kat_scalar(cid, 12345, 6789, scal, nthreads=16) % r
ok = (co.jac_to_affine(cid, out) == co.jac_to_affine(cid, co.gen_mul(cid, k))).all()
print(f"2^{log_n} {curve} KAT {'ok' if ok else 'MISMATCH'}", flush=True)
sys.exit(0 if ok else 1)
