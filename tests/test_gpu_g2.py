"""GPU parity tests of the G2 (Fq2) paths: MSM (field2.cl), the
batched MSM and the EC-FFT instantiated over G2.  Checker: the pure-Python
G2 restatement (tests/golden/msm_*_g2.npz, pinned by test_oracle_g2.py) and
known answers built from the public generator:  P_i = (a + i b) G2  =>
sum s_i P_i = (sum s_i (a + i b) mod r) G2."""
import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po
from conftest import load_npz

pytestmark = pytest.mark.gpu

G2 = [("bls12_381_g2", 2, po.BLS12_381_G2), ("bn254_g2", 3, po.BN254_G2)]


def to_py_affine(cv, jac):
    """normalised Jacobian u64 limbs ([c0, c1] per coordinate) -> Python affine or None."""
    n = cv.fq.limbs64
    p = cv.fq.modulus
    j = np.asarray(jac).reshape(3, 2 * n)

    def fq2(l):
        return po.Fq2(cv.fq.from_mont(po.limbs_to_int(l[:n])), cv.fq.from_mont(po.limbs_to_int(l[n:])), p)

    X, Y, Z = fq2(j[0]), fq2(j[1]), fq2(j[2])
    return po.jac_to_affine((X, Y, Z), p)


def fq2_limbs(cv, a):
    n = cv.fq.limbs64
    return po.int_to_limbs(cv.fq.to_mont(a.c0), n) + po.int_to_limbs(cv.fq.to_mont(a.c1), n)


@pytest.mark.parametrize("cname,cid,cv", G2)
def test_g2_msm_golden(gpu_programs, cname, cid, cv):
    progs, devs = gpu_programs
    k = ecgpu.MultiexpKernel.create(progs, devs, cname)
    g = load_npz(f"msm_{cname}.npz")
    pool = ecgpu.Worker()
    n = cv.fq.limbs64
    for i, _ in enumerate(g["cases"]):
        out = k.multiexp(pool, g[f"bases_{i}"], g[f"exps_{i}"], 0)
        got = to_py_affine(cv, out)
        if g[f"inf_{i}"][0]:
            assert got is None
        else:
            o = g[f"out_{i}"]
            assert got is not None and fq2_limbs(cv, got[0]) + fq2_limbs(cv, got[1]) == [int(v) for v in o], i


@pytest.mark.parametrize("cname,cid,cv", G2)
def test_g2_msm_kat_2p20(gpu_programs, cname, cid, cv):
    prog = gpu_programs[0][0]
    n = 1 << 20
    a, b = 0x5EED, 0x1234567
    d_b = ecgpu.gen_bases_dev(prog, cname, a, b, n)
    # spot-check the generated bases against (a + i b) G2
    host_b = d_b.read(shape=(n, 4 * cv.fq.limbs64))
    for i in (0, 1, 63, 64, n - 1):
        P = po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, (a + i * b) % cv.fr.modulus))
        assert [int(v) for v in host_b[i]] == fq2_limbs(cv, P[0]) + fq2_limbs(cv, P[1])
    rng = np.random.default_rng(20 + cid)
    E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    E[:, 3] &= np.uint64((1 << (cv.fr.bits - 192 - 1)) - 1)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    out = ecgpu.msm_dev(prog, cname, d_b, d_e, n)
    kat = co.kat_scalar(cid - 2, a, b, E, nthreads=16)  # scalar-side identity: same r as G1
    want = po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, kat))
    assert to_py_affine(cv, out) == want


@pytest.mark.parametrize("cname,cid,cv", G2)
def test_g2_multiple_multiexp(gpu_programs, cname, cid, cv):
    prog = gpu_programs[0][0]
    L, lines, chunks = 64, 2, 4
    a, b = 99, 7
    d_b = ecgpu.gen_bases_dev(prog, cname, a, b, L * lines)
    rng = po.Xoshiro256ss(3)
    exps = co.u64arr([rng.field_element(cv.fr) for _ in range(L)], 4)
    got = ecgpu.multiple_multiexp(prog, d_b, exps, chunks, curve=cname)
    r = cv.fr.modulus
    clen = L // chunks
    for t in range(lines * chunks):
        l, c = divmod(t, chunks)
        k = sum(po.limbs_to_int(exps[c * clen + i]) * (a + (l * L + c * clen + i) * b) for i in range(clen)) % r
        assert to_py_affine(cv, got[t]) == po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, k)), t


@pytest.mark.parametrize("cname,cid,cv", G2)
def test_g2_ec_fft_linearity(gpu_programs, cname, cid, cv):
    """P_j = (a + j b) G2 => EC-FFT(P)_k = FFT(a + j b)_k G2."""
    prog = gpu_programs[0][0]
    log_n = 8
    n = 1 << log_n
    a, b = 11, 5
    d_b = ecgpu.gen_bases_dev(prog, cname, a, b, n)
    aff = d_b.read(shape=(n, 4 * cv.fq.limbs64))
    one = fq2_limbs(cv, po.Fq2(1, 0, cv.fq.modulus))
    jac = np.ascontiguousarray(np.concatenate([aff, np.tile(np.array(one, dtype=np.uint64), (n, 1))], axis=1))
    r = cv.fr.modulus
    w = cv.fr.omega(n)
    k = ecgpu.EcFftKernel.create([prog], cname)
    k.radix_ec_fft(jac, co.u64arr([cv.fr.to_mont(w)], 4)[0], log_n)
    fs = po.serial_fft([(a + j * b) % r for j in range(n)], w, log_n, r)
    for kk in (0, 1, 2, 100, n - 1):
        assert to_py_affine(cv, jac[kk]) == po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, fs[kk])), kk


@pytest.mark.parametrize("cname,cid,cv", G2)
def test_g2_ec_fft_equal_and_alternating_points(gpu_programs, cname, cid, cv):
    """All P_j = P: out_0 = n P and out_k = O for k != 0 (sum_j w^(jk) = 0);
    P_j = (-1)^j P: out_(n/2) = n P, every other out_k = O.  Stage 0 adds P to
    P and to -P, so the full add's doubling and identity branches run (on lane
    pairs, curve_rr2.hpp rr_add_x2, at these sizes)."""
    prog = gpu_programs[0][0]
    p = cv.fq.modulus
    r = cv.fr.modulus
    k0 = 0xBEEF + cid
    P = po.g2_scalar_mul(cv, cv.gen, k0)
    Pa = po.g2_to_affine(cv, P)
    one = fq2_limbs(cv, po.Fq2(1, 0, p))
    row = np.array(fq2_limbs(cv, Pa[0]) + fq2_limbs(cv, Pa[1]) + one, dtype=np.uint64)
    nrow = np.array(fq2_limbs(cv, Pa[0]) + fq2_limbs(cv, po.Fq2(0, 0, p) - Pa[1]) + one, dtype=np.uint64)
    k = ecgpu.EcFftKernel.create([prog], cname)
    for log_n in (1, 3, 6):
        n = 1 << log_n
        om = co.u64arr([cv.fr.to_mont(cv.fr.omega(n))], 4)[0]
        nP = po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, n * k0 % r))
        for pattern, hot in (("equal", 0), ("alternating", n // 2)):
            rows = [row if (pattern == "equal" or j % 2 == 0) else nrow for j in range(n)]
            jac = np.ascontiguousarray(np.stack(rows))
            k.radix_ec_fft(jac, om, log_n)
            for kk in range(n):
                got = to_py_affine(cv, jac[kk])
                if kk == hot:
                    assert got == nP, (log_n, pattern, kk)
                else:
                    assert got is None, (log_n, pattern, kk)


@pytest.mark.parametrize("cname,cid,cv", G2)
def test_g2_msm_exceptional_paths(gpu_programs, cname, cid, cv):
    """Equal bases drive the doubling branch of the mixed add (acc = P, + P)
    and of the full add in the combine / reduction (k P + k P); a base next to
    its negative drives the P + (-P) = O branch.  The reduced-radix Fq2 form
    detects both on PP's components (curve_rr2.hpp); random inputs never do."""
    prog = gpu_programs[0][0]
    p = cv.fq.modulus
    r = cv.fr.modulus
    k0 = 0xC0FFEE
    P = po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, k0))
    row = np.array(fq2_limbs(cv, P[0]) + fq2_limbs(cv, P[1]), dtype=np.uint64)
    nrow = np.array(fq2_limbs(cv, P[0]) + fq2_limbs(cv, po.Fq2(0, 0, p) - P[1]), dtype=np.uint64)
    rng = np.random.default_rng(7 + cid)
    for n in (64, 1 << 16):
        B = np.ascontiguousarray(np.tile(row, (n, 1)))
        E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
        E[:, 3] &= np.uint64((1 << (cv.fr.bits - 192 - 1)) - 1)
        d_b = ecgpu.DeviceBuffer.upload(prog, B)
        d_e = ecgpu.DeviceBuffer.upload(prog, E)
        got = to_py_affine(cv, ecgpu.msm_dev(prog, cname, d_b, d_e, n))
        s = sum(po.limbs_to_int(e) for e in E) % r
        assert got == po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, s * k0 % r)), n
        # equal scalars, one base and its negative alternating: every bucket cancels
        Bn = np.ascontiguousarray(np.where((np.arange(n) % 2 == 1)[:, None], nrow, row))
        Ee = np.ascontiguousarray(np.tile(E[0], (n, 1)))
        d_b = ecgpu.DeviceBuffer.upload(prog, Bn)
        d_e = ecgpu.DeviceBuffer.upload(prog, Ee)
        assert to_py_affine(cv, ecgpu.msm_dev(prog, cname, d_b, d_e, n)) is None, n
