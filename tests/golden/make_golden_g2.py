"""Mint the G2 MSM fixtures (tests/golden/msm_<curve>_g2.npz) from the pure-Python
restatement (oracle/py_oracle.py: multiexp_cpu over Fq2, multiexp_cpu.rs:244-367).
Bases are k_i * G2 for seeded k_i; edge scalars 0, 1, r-1 and a repeated base
are included.  Layout = the C ABI's: coordinates [c0, c1] Montgomery u64 limbs.
Run from the repo root: python3 tests/golden/make_golden_g2.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import py_oracle as po  # noqa: E402


def fq2_limbs(cv, a):
    n = cv.fq.limbs64
    return po.int_to_limbs(cv.fq.to_mont(a.c0), n) + po.int_to_limbs(cv.fq.to_mont(a.c1), n)


def main():
    for cv in po.CURVES_G2.values():
        rng = po.Xoshiro256ss(0x62 + len(cv.name))
        out = {}
        cases = [1, 5, 33, 100]
        for k, n in enumerate(cases):
            ks = [rng.field_element(cv.fr) for _ in range(n)]
            bases = [po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, kk)) for kk in ks]
            exps = [rng.field_element(cv.fr) for _ in range(n)]
            if n >= 5:
                exps[0], exps[1], exps[2] = 0, 1, cv.fr.modulus - 1
                bases[4] = bases[3]  # repeated base
            res = po.g2_to_affine(cv, po.g2_multiexp_cpu(cv, bases, exps))
            out[f"bases_{k}"] = np.array([fq2_limbs(cv, b[0]) + fq2_limbs(cv, b[1]) for b in bases], dtype=np.uint64)
            out[f"exps_{k}"] = np.array([po.int_to_limbs(e, 4) for e in exps], dtype=np.uint64)
            out[f"inf_{k}"] = np.array([res is None], dtype=bool)
            out[f"out_{k}"] = np.array(fq2_limbs(cv, res[0]) + fq2_limbs(cv, res[1]) if res else [0] * (4 * cv.fq.limbs64),
                                       dtype=np.uint64)
        out["cases"] = np.array(cases)
        path = os.path.join(ROOT, "tests", "golden", f"msm_{cv.name}.npz")
        np.savez_compressed(path, **out)
        print("wrote", path)


if __name__ == "__main__":
    main()
