"""CPU checks of the G2 restatement (oracle/py_oracle.py Fq2 / CurveG2) that
pins tests/golden/msm_*_g2.npz.  The reference's Fp2 is ag-build/cl/
field2.cl:1-61 (u^2 = -1); curve constants are the public BLS12-381 / BN254
G2 definitions (ark-bls12-381 / ark-bn254 0.4, absent here)."""
import numpy as np
import pytest

import py_oracle as po
from conftest import load_npz

G2 = list(po.CURVES_G2.values())


@pytest.mark.parametrize("cv", G2, ids=lambda c: c.name)
def test_g2_generator_and_order(cv):
    G = cv.gen
    assert po.on_curve_g2(cv, G)
    assert po.g2_scalar_mul(cv, G, cv.fr.modulus)[2] == 0          # r G = O
    assert po.g2_to_affine(cv, po.g2_scalar_mul(cv, G, cv.fr.modulus + 1)) == G


@pytest.mark.parametrize("cv", G2, ids=lambda c: c.name)
def test_fq2_arithmetic(cv):
    p = cv.fq.modulus
    u = po.Fq2(0, 1, p)
    assert u * u == p - 1                                              # u^2 = -1
    a, b = po.Fq2(123456789, 987654321, p), po.Fq2(p - 5, 77, p)
    assert (a * b) * (b ** -1) == a
    assert (a + b) - b == a and a * (b + 1) == a * b + a


@pytest.mark.parametrize("cv", G2, ids=lambda c: c.name)
def test_g2_multiexp_cpu_vs_naive(cv):
    rng = po.Xoshiro256ss(7)
    n = 20
    bases = [po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, rng.field_element(cv.fr))) for _ in range(n)]
    exps = [rng.field_element(cv.fr) for _ in range(n)]
    exps[3] = 1
    a = po.g2_to_affine(cv, po.g2_multiexp_cpu(cv, bases, exps))
    b = po.g2_to_affine(cv, po.naive_multiexp(cv, bases, exps))
    assert a == b


@pytest.mark.parametrize("cv", G2, ids=lambda c: c.name)
def test_g2_golden_fixture_consistent(cv):
    """The committed fixture's smallest cases re-derived here."""
    g = load_npz(f"msm_{cv.name}.npz")
    n = cv.fq.limbs64
    p = cv.fq.modulus

    def fq2(limbs):
        return po.Fq2(cv.fq.from_mont(po.limbs_to_int(limbs[:n])), cv.fq.from_mont(po.limbs_to_int(limbs[n:2 * n])), p)

    for k in (0, 1):
        B = g[f"bases_{k}"]
        bases = [(fq2(r[:2 * n]), fq2(r[2 * n:])) for r in B]
        exps = [po.limbs_to_int(e) for e in g[f"exps_{k}"]]
        for b in bases:
            assert po.on_curve_g2(cv, b)
        res = po.g2_to_affine(cv, po.g2_multiexp_cpu(cv, bases, exps))
        o = g[f"out_{k}"]
        assert res == (fq2(o[:2 * n]), fq2(o[2 * n:]))
