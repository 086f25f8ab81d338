#!/usr/bin/env python3
"""Mint the golden fixtures under tests/golden/ from the pure-Python big-int
restatement (oracle/py_oracle.py) of the reference's serial_fft and
multiexp_cpu.  The reference itself cannot run here (Rust workspace; no
cargo/rustc in the image) and holds no fixtures of its own, so these vectors
are generated from the restatement and cross-checked against the reference's
own property tests (naive multiexp == multiexp_cpu, serial == naive DFT).

    python3 tests/golden/make_golden.py      # rewrites the .npz fixtures

Fixtures (numpy .npz, no pickles):
  fft_<field>.npz   log_n 1..10: in_<k>, out_<k> (n x 4 Montgomery), omega_<k>
  fft_bls12_381_fr_2p16.json   config (1): sha256 of serial_fft output at 2^16
  msm_<curve>.npz   cases: bases_<k> (N x 2Lq), exps_<k> (N x 4 canonical),
                    out_<k> (2Lq affine Montgomery, zeros = identity), inf_<k>
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import py_oracle as po  # noqa: E402


def limbs(vals, n):
    out = np.zeros((len(vals), n), dtype=np.uint64)
    for k, v in enumerate(vals):
        for i in range(n):
            out[k, i] = (v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return out


def fft_fixtures():
    for f in (po.BLS12_381_FR, po.BN254_FR):
        arrays = {}
        for log_n in range(1, 11):
            n = 1 << log_n
            rng = po.Xoshiro256ss(0x0FF70016 ^ (log_n << 8) ^ f.limbs64)
            xs = [rng.field_element(f) for _ in range(n)]
            if log_n == 3:
                xs[0] = 0
                xs[1] = f.modulus - 1
            w = f.omega(n)
            ys = po.serial_fft(xs, w, log_n, f.modulus)
            if log_n <= 6:
                assert ys == po.naive_dft(xs, w, f.modulus)
            arrays[f"in_{log_n}"] = limbs([f.to_mont(x) for x in xs], 4)
            arrays[f"out_{log_n}"] = limbs([f.to_mont(y) for y in ys], 4)
            arrays[f"omega_{log_n}"] = limbs([f.to_mont(w)], 4)[0]
        np.savez_compressed(os.path.join(HERE, f"fft_{f.name}.npz"), **arrays)


def fft_2p16_hash():
    f = po.BLS12_381_FR
    log_n = 16
    n = 1 << log_n
    rng = po.Xoshiro256ss(0x0FF70016)
    xs = [rng.field_element(f) for _ in range(n)]
    ys = po.serial_fft(xs, f.omega(n), log_n, f.modulus)
    inp = limbs([f.to_mont(x) for x in xs], 4)
    out = limbs([f.to_mont(y) for y in ys], 4)
    meta = {"config": "BLS12-381 Fr radix-2 FFT at 2^16 on serial_fft (BASELINE config 1)",
            "seed": "xoshiro256** 0x0FF70016", "log_n": log_n,
            "input_sha256": hashlib.sha256(inp.tobytes()).hexdigest(),
            "output_sha256": hashlib.sha256(out.tobytes()).hexdigest()}
    with open(os.path.join(HERE, "fft_bls12_381_fr_2p16.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


def gen_bases(cv, a, b, n):
    """P_i = (a + i b) G by repeated addition, normalised to affine."""
    p = cv.fq.modulus
    P = po.scalar_mul((cv.gx, cv.gy), a, p)
    Q = po.jac_to_affine(po.scalar_mul((cv.gx, cv.gy), b, p), p)
    out = []
    for _ in range(n):
        out.append(po.jac_to_affine(P, p))
        P = po.jac_add_mixed(P, Q, p)
    return out


def msm_fixtures():
    for cv in (po.BLS12_381, po.BN254):
        fq, fr = cv.fq, cv.fr
        nq = fq.limbs64
        r = fr.modulus
        arrays = {}
        cases = [1, 2, 3, 5, 31, 32, 33, 100, 257, 1024]
        for k, n in enumerate(cases):
            rng = po.Xoshiro256ss(0x35A00020 ^ (k << 12) ^ nq)
            bases = gen_bases(cv, 1000 + 17 * k, 7 + k, n)
            exps = [rng.field_element(fr) for _ in range(n)]
            if n >= 5:
                exps[0] = 0
                exps[1] = 1
                exps[2] = r - 1
                exps[3] = (1 << (fr.bits - 1)) - 1   # all-ones low windows
                exps[4] = 1 << (fr.bits - 1)         # top bit only
            if n >= 31:
                bases[10] = bases[9]                 # repeated base -> P + P (doubling path)
                exps[10] = exps[9]
                bases[12] = bases[11]
                exps[12] = (r - exps[11]) % r        # s P + (r - s) P = O contributions
            if n >= 100:
                bases[50] = None                     # identity base with zero scalar (allowed)
                exps[50] = 0
            ref = po.multiexp_cpu(cv, bases, exps)
            if n <= 100:
                assert po.jac_eq(ref, po.naive_multiexp(cv, bases, exps), fq.modulus)
            aff = po.jac_to_affine(ref, fq.modulus)
            arrays[f"bases_{k}"] = limbs([fq.to_mont(c) if b is not None else 0
                                          for b in bases for c in (b if b is not None else (0, 0))],
                                         nq).reshape(n, 2 * nq)
            arrays[f"exps_{k}"] = limbs(exps, 4)
            arrays[f"out_{k}"] = (limbs([fq.to_mont(aff[0]), fq.to_mont(aff[1])], nq).reshape(2 * nq)
                                  if aff is not None else np.zeros(2 * nq, dtype=np.uint64))
            arrays[f"inf_{k}"] = np.array([aff is None])
        arrays["cases"] = np.array(cases, dtype=np.int64)
        np.savez_compressed(os.path.join(HERE, f"msm_{cv.name}.npz"), **arrays)


if __name__ == "__main__":
    fft_fixtures()
    fft_2p16_hash()
    msm_fixtures()
    print("fixtures written to", HERE)
