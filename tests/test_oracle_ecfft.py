"""CPU checks of the EC-FFT oracle (oracle.c orc_serial_ec_fft, a restatement
of serial_ec_fft, ec-gpu-proxy/src/ec_fft_cpu.rs:12-56).

The reference pins its EC-FFT against arkworks' Radix2EvaluationDomain::fft
(tests/ec_fft.rs:33-82, ag-cuda-ec/src/ec_fft.rs:97-131), which is not
available here.  The oracle is pinned instead by
  * the DFT definition, out_k = sum_j omega^(jk) P_j (O(n^2) scalar mults),
  * linearity through the scalar FFT: for P_j = s_j G,
    EC-FFT(P)_k = (FFT(s)_k) G, with the scalar FFT itself pinned by the
    golden vectors (test_oracle.py)."""
import numpy as np
import pytest

import coracle as co
import py_oracle as po

CURVES = [("bls12_381", 0), ("bn254", 1)]


def points_from_scalars(cid, scalars):
    return np.stack([co.gen_mul(cid, s) for s in scalars])  # Jacobian, Z != 1 in general


def same_points(cid, a, b):
    for k, (p, q) in enumerate(zip(a, b)):
        x, y = co.jac_to_affine(cid, p), co.jac_to_affine(cid, q)
        if (x is None) != (y is None) or (x is not None and not (x == y).all()):
            return False
    return True


@pytest.mark.parametrize("cname,cid", CURVES)
def test_ec_fft_oracle_matches_dft_definition(cname, cid):
    cv = po.CURVES[cname]
    rng = po.Xoshiro256ss(900 + cid)
    for log_n in range(0, 5):
        n = 1 << log_n
        pts = points_from_scalars(cid, [rng.field_element(cv.fr) for _ in range(n)])
        om = co.u64arr([cv.fr.to_mont(cv.fr.omega(n))], 4)[0]
        got = co.serial_ec_fft(cid, pts, om, log_n)
        want = co.naive_ec_dft(cid, pts, om, log_n)
        assert same_points(cid, got, want), log_n


@pytest.mark.parametrize("cname,cid", CURVES)
def test_ec_fft_oracle_linearity_kat(cname, cid):
    """P_j = s_j G  =>  EC-FFT(P)_k = FFT(s)_k G (scalar FFT: py_oracle.serial_fft)."""
    cv = po.CURVES[cname]
    r = cv.fr.modulus
    rng = po.Xoshiro256ss(77 + cid)
    log_n = 6
    n = 1 << log_n
    s = [rng.field_element(cv.fr) for _ in range(n)]
    s[5] = 0  # an identity input
    pts = points_from_scalars(cid, s)
    w = cv.fr.omega(n)
    got = co.serial_ec_fft(cid, pts, co.u64arr([cv.fr.to_mont(w)], 4)[0], log_n, nthreads=4)
    fs = po.serial_fft(list(s), w, log_n, r)
    want = points_from_scalars(cid, fs)
    assert same_points(cid, got, want)
    # thread count does not change the result
    got1 = co.serial_ec_fft(cid, pts, co.u64arr([cv.fr.to_mont(w)], 4)[0], log_n, nthreads=1)
    assert same_points(cid, got, got1)
