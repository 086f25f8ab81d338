"""Per-rank work of the two N-GPU MSM splits, measured on ONE GPU (dev tool).

For N in {2, 4, 8}: every rank's local step is run in turn on the same
device and timed -- range split (ecg_msm_dev on the rank's n/N shard, a view
of the prepared buffer) and grid split (ecg_msm_grid_part over all n terms,
1/N of the (window x term) grid).  The slowest rank's time is what an N-GPU
step costs before the partial exchange (~40-70 us over RCCL).  The grid
partials are folded and checked against the single-GPU msm_dev result.

Usage: python tools/grid_split_probe.py [log_n] [curve] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ecgpu  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
curve = sys.argv[2] if len(sys.argv) > 2 else "bls12_381"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cid = ecgpu.CURVE_NAMES[curve]
n = 1 << log_n
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(11)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
E[:, 3] &= np.uint64(2**60 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
d_raw = ecgpu.gen_bases_dev(prog, curve, 12345, 678910, n)
prep = ecgpu.prepare_bases(prog, curve, d_raw, n)
d_raw.free()


def timed(fn):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, out


full_ms, want = timed(lambda: ecgpu.msm_dev(prog, curve, prep, d_e, n))
import coracle as co  # noqa: E402  (checker only: folds the partials)

want_aff = co.jac_to_affine(cid, want)
print(json.dumps({"n": n, "curve": curve, "single_gpu_ms": full_ms}), flush=True)


class _Ptr:
    def __init__(self, buf, off):
        import ctypes
        self.ptr = ctypes.c_void_p(buf.ptr.value + off)


for N in (2, 4, 8):
    rng_ms, grid_ms, pieces = [], [], []
    parts = []
    for r in range(N):
        i0, i1 = r * n // N, (r + 1) * n // N
        ms, _ = timed(lambda: ecgpu.msm_dev(prog, curve, prep.view(i0, i1 - i0), _Ptr(d_e, i0 * 32), i1 - i0))
        rng_ms.append(ms)
        ms, (part, k) = timed(lambda: ecgpu.msm_grid_part(prog, curve, prep, d_e, n, r, N))
        grid_ms.append(ms)
        pieces.append(k)
        parts.append(part)
    acc = np.zeros(3 * ecgpu.CURVE_FQ_LIMBS[cid], dtype=np.uint64)
    for p in parts:
        co.lib().orc_jac_add(cid, co.ptr(acc), co.ptr(acc), co.ptr(np.ascontiguousarray(p)))
    ok = bool((co.jac_to_affine(cid, acc) == want_aff).all())
    print(json.dumps({"N": N, "range_ms": rng_ms, "grid_ms": grid_ms, "grid_pieces": pieces,
                      "range_max_ms": max(rng_ms), "grid_max_ms": max(grid_ms),
                      "range_eff": full_ms / N / max(rng_ms), "grid_eff": full_ms / N / max(grid_ms),
                      "grid_fold_equals_single": ok}), flush=True)
    if not ok:
        sys.exit(1)
