"""Quick end-to-end GPU parity probe (dev tool): HIP path vs the C oracle."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import coracle as co  # noqa: E402
import py_oracle as po  # noqa: E402
import ecgpu  # noqa: E402


def rand_fr(rng, f, n):
    return co.u64arr([f.to_mont(rng.field_element(f)) for _ in range(n)], 4)


def main():
    rng = po.Xoshiro256ss(7)
    devs = ecgpu.Device.all()
    print("devices:", len(devs))
    progs = [ecgpu.program(d) for d in devs[:1]]
    for fname, fid in (("bls12_381_fr", 0), ("bn254_fr", 2)):
        f = po.FIELDS[fname]
        k = ecgpu.FftKernel.create(progs, fname)
        for log_n in list(range(1, 13)) + [16, 18]:
            n = 1 << log_n
            a = rand_fr(rng, f, min(n, 4096))
            if n > 4096:
                a = np.tile(a, (n // 4096, 1))
                a = np.ascontiguousarray(a)
            om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
            ref = co.serial_fft(fid, a, om, log_n) if log_n <= 12 else co.parallel_fft(fid, a, om, log_n, 3)
            g = a.copy()
            t = time.time()
            k.radix_fft(g, om, log_n)
            dt = time.time() - t
            ok = (g == ref).all()
            print(f"fft {fname} 2^{log_n}: {'OK' if ok else 'MISMATCH'} ({dt*1e3:.1f} ms)")
            if not ok:
                bad = np.nonzero((g != ref).any(axis=1))[0]
                print("   first bad idx", bad[:8], "count", len(bad))
    for cname, cid in (("bls12_381", 0), ("bn254", 1)):
        cv = po.CURVES[cname]
        mk = ecgpu.MultiexpKernel.create(progs, devs, cname)
        for n in (1, 2, 3, 17, 64, 1000, 4096, 1 << 14):
            B = co.gen_bases(cid, 12345 + n, 6789, n, 8)
            E = co.u64arr([rng.field_element(cv.fr) for _ in range(n)], 4)
            if n > 2:
                E[0] = 0
                E[1] = [1, 0, 0, 0]
            t = time.time()
            got = mk.multiexp(ecgpu.Worker(), B, E, 0)
            dt = time.time() - t
            ref = co.multiexp_cpu(cid, B, E, nthreads=8)
            ra = co.jac_to_affine(cid, ref)
            ga = co.jac_to_affine(cid, got)
            ok = (ra is None and ga is None) or (ra is not None and ga is not None and (ra == ga).all())
            print(f"msm {cname} n={n}: {'OK' if ok else 'MISMATCH'} ({dt*1e3:.1f} ms)")
    print("done")


if __name__ == "__main__":
    main()
