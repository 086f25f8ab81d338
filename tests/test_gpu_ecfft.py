"""GPU parity tests of the G1 EC-FFT (ecg_ec_fft / EcFftKernel mirror).

Model: ec-gpu-proxy/tests/ec_fft.rs gpu_ec_fft_consistency (log_d 1..=16,
random points, compared with a CPU FFT as group elements) and
gpu_ec_fft_many_consistency (three inputs per call), ag-cuda-ec/src/ec_fft.rs
test_ec_fft (degrees 4..8, omegas = [w, w^2, w^4, ...]).  Checker: the oracle's
serial_ec_fft restatement (tests/test_oracle_ecfft.py pins it), and at the
largest sizes the linearity known answer  P_j = s_j G  =>  out_k = FFT(s)_k G."""
import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po

pytestmark = pytest.mark.gpu

CURVES = [("bls12_381", 0), ("bn254", 1)]


def jac_from_affine(cv, aff):
    """(n, 2 Lq) affine Montgomery -> (n, 3 Lq) Jacobian with Z = 1."""
    one = co.u64arr([cv.fq.to_mont(1)], cv.fq.limbs64)[0]
    z = np.tile(one, (aff.shape[0], 1))
    return np.ascontiguousarray(np.concatenate([aff, z], axis=1))


def omega_m(cv, n):
    return co.u64arr([cv.fr.to_mont(cv.fr.omega(n))], 4)[0]


def same_points(cid, a, b):
    for k, (p, q) in enumerate(zip(a, b)):
        x, y = co.jac_to_affine(cid, p), co.jac_to_affine(cid, q)
        if (x is None) != (y is None) or (x is not None and not (x == y).all()):
            return False
    return True


def normalised(cv, pts):
    lq = cv.fq.limbs64
    one = cv.fq.to_mont(1)
    for p in pts:
        j = co.to_ints(p.reshape(3, lq))
        if not (j[2] == one or j == [0, one, 0]):
            return False
    return True


@pytest.fixture(scope="module")
def kernels(gpu_programs):
    progs, _ = gpu_programs
    return {name: ecgpu.EcFftKernel.create(progs, name) for name, _ in CURVES}


@pytest.fixture
def radix():
    """ecg_ec_fft_set_radix for one test, back to automatic afterwards."""
    yield ecgpu.ec_fft_set_radix
    ecgpu.ec_fft_set_radix(0)


@pytest.mark.parametrize("max_radix", [0, 1, 3, 8], ids=["auto", "radix2", "radix8", "radix256"])
@pytest.mark.parametrize("cname,cid", CURVES)
def test_gpu_ec_fft_consistency(kernels, radix, cname, cid, max_radix):
    """tests/ec_fft.rs:33-82: log_d 1..=14 against serial_ec_fft, through every
    stage form: the engine's choice, radix-2 stages only, and radix-2^d stages
    of at most 2^3 and 2^8 (ecfft_rprod / ecfft_rsum kernels; mixed radices
    where d does not divide log_d)."""
    radix(max_radix)
    cv = po.CURVES[cname]
    top = 14 if cid == 0 else 12
    for log_d in range(1, top + 1):
        n = 1 << log_d
        pts = jac_from_affine(cv, co.gen_bases(cid, 1000 + log_d, 7919, n))
        om = omega_m(cv, n)
        want = co.serial_ec_fft(cid, pts, om, log_d, nthreads=16)
        got = pts.copy()
        kernels[cname].radix_ec_fft_many([got], [om], [log_d])
        assert normalised(cv, got[:64])
        assert same_points(cid, got, want), log_d


@pytest.mark.parametrize("cname,cid", CURVES)
def test_gpu_ec_fft_large_kat(kernels, cname, cid):
    """log_d 15, 16 (the reference test's top sizes): P_j = (a + j b) G, so
    out_k = FFT(a + j b)_k G; all outputs compared against a device MSM-free
    CPU check on a sample of k plus the full scalar FFT."""
    cv = po.CURVES[cname]
    r = cv.fr.modulus
    a, b = 31337, 271828
    for log_d in (15, 16):
        n = 1 << log_d
        pts = jac_from_affine(cv, co.gen_bases(cid, a, b, n, nthreads=16))
        w = cv.fr.omega(n)
        got = pts.copy()
        kernels[cname].radix_ec_fft(got, co.u64arr([cv.fr.to_mont(w)], 4)[0], log_d)
        sc = co.u64arr([cv.fr.to_mont((a + j * b) % r) for j in range(n)], 4)
        fs = co.from_mont(2 * cid, co.serial_fft(2 * cid, sc, co.u64arr([cv.fr.to_mont(w)], 4)[0], log_d))
        fs = co.to_ints(fs)
        for k in list(range(0, n, 997)) + [1, 2, n // 2, n - 1]:
            want = co.jac_to_affine(cid, co.gen_mul(cid, fs[k]))
            g = co.jac_to_affine(cid, got[k])
            assert (g is None and want is None) or (g == want).all(), (log_d, k)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_gpu_ec_fft_many_and_unnormalised_inputs(kernels, cname, cid):
    """tests/ec_fft.rs:84-170 (three inputs per call) with Jacobian inputs of
    arbitrary Z and identity elements (Z = 0)."""
    cv = po.CURVES[cname]
    rng = po.Xoshiro256ss(555 + cid)
    lq = cv.fq.limbs64
    ins, oms, lns, wants = [], [], [], []
    for log_d in (3, 7, 10):
        n = 1 << log_d
        if log_d == 10:
            pts = jac_from_affine(cv, co.gen_bases(cid, 17, 19, n))
        else:
            pts = np.stack([co.gen_mul(cid, rng.field_element(cv.fr)) for _ in range(n)])  # Z != 1
        pts[1] = 0
        pts[1, lq:2 * lq] = co.u64arr([cv.fq.to_mont(1)], lq)[0]  # (0, 1, 0)
        pts[2, 2 * lq:] = 0  # Z = 0 with junk X, Y: still the identity
        om = omega_m(cv, n)
        ins.append(np.ascontiguousarray(pts))
        oms.append(om)
        lns.append(log_d)
        wants.append(co.serial_ec_fft(cid, pts, om, log_d, nthreads=16))
    kernels[cname].radix_ec_fft_many(ins, oms, lns)
    for g, w in zip(ins, wants):
        assert same_points(cid, g, w)


@pytest.mark.parametrize("max_radix", [0, 1], ids=["auto", "radix2"])
@pytest.mark.parametrize("cname,cid", CURVES)
def test_gpu_ec_fft_equal_and_opposite_points(kernels, radix, cname, cid, max_radix):
    """Inputs whose butterflies add a point to itself and to its negative: all
    P_j equal (stage 0 computes P + P and P - P), and P_j = (-1)^j P.  These
    take the doubling and identity branches of the full add (on G1 the lane-pair
    form, curve_rr.hpp rr_add_x2), against serial_ec_fft."""
    radix(max_radix)
    cv = po.CURVES[cname]
    lq = cv.fq.limbs64
    for log_d in (1, 4, 6):
        n = 1 << log_d
        P = co.gen_mul(cid, 987654321 + cid)
        negP = co.gen_mul(cid, (cv.fr.modulus - 987654321 - cid) % cv.fr.modulus)
        for pattern in ("equal", "alternating"):
            if pattern == "equal":
                pts = np.tile(P, (n, 1))
            else:
                pts = np.stack([P if j % 2 == 0 else negP for j in range(n)])
            pts = np.ascontiguousarray(pts.reshape(n, 3 * lq))
            om = omega_m(cv, n)
            want = co.serial_ec_fft(cid, pts, om, log_d, nthreads=16)
            got = pts.copy()
            kernels[cname].radix_ec_fft(got, om, log_d)
            assert same_points(cid, got, want), (log_d, pattern)


def test_ag_cuda_ec_radix_ec_fft(gpu_programs):
    """ag-cuda-ec/src/ec_fft.rs:97-131: degrees 4..8, omegas[i] = omega^(2^i)."""
    prog = gpu_programs[0][0]
    cv = po.CURVES["bls12_381"]
    r = cv.fr.modulus
    for degree in range(4, 9):
        n = 1 << degree
        w = cv.fr.omega(n)
        omegas = co.u64arr([cv.fr.to_mont(pow(w, 1 << i, r)) for i in range(32)], 4)
        pts = jac_from_affine(cv, co.gen_bases(0, 5 + degree, 3, n))
        want = co.serial_ec_fft(0, pts, omegas[0], degree, nthreads=16)
        got = pts.copy()
        ecgpu.radix_ec_fft(prog, got, omegas)
        assert same_points(0, got, want), degree


def test_gpu_ec_fft_edges(kernels, gpu_programs):
    cv = po.CURVES["bls12_381"]
    lq = cv.fq.limbs64
    k = kernels["bls12_381"]
    # log_n = 0: the input, normalised
    p = co.gen_mul(0, 123456789).reshape(1, 3 * lq).copy()
    q = p.copy()
    k.radix_ec_fft(q, omega_m(cv, 1), 0)
    assert same_points(0, q, p) and normalised(cv, q)
    # beyond the two-adicity (BLS12-381 Fr: 32) -> error before any copy
    with pytest.raises(ecgpu.EcError):
        lib = ecgpu.lib()
        h = gpu_programs[0][0].handle
        dummy = np.zeros(3 * lq, dtype=np.uint64)
        ecgpu._check(lib.ecg_ec_fft(h, 0, ecgpu._ptr(dummy), ecgpu._ptr(omega_m(cv, 2)), 33,
                                    ecgpu.ABORT_CB(0), None))
    # shape mismatch
    with pytest.raises(ecgpu.EcError):
        k.radix_ec_fft(np.zeros((8, 3 * lq), dtype=np.uint64), omega_m(cv, 16), 4)
    # all-identity input stays the identity
    z = np.zeros((16, 3 * lq), dtype=np.uint64)
    k.radix_ec_fft(z, omega_m(cv, 16), 4)
    one = cv.fq.to_mont(1)
    assert all(co.to_ints(row.reshape(3, lq)) == [0, one, 0] for row in z)


def test_gpu_ec_fft_abort(gpu_programs):
    progs, _ = gpu_programs
    k = ecgpu.EcFftKernel.create_with_abort(progs, lambda: True)
    cv = po.CURVES["bls12_381"]
    pts = jac_from_affine(cv, co.gen_bases(0, 1, 1, 16))
    with pytest.raises(ecgpu.Aborted):
        k.radix_ec_fft(pts, omega_m(cv, 16), 4)


def test_gpu_ec_fft_device_resident(gpu_programs):
    prog = gpu_programs[0][0]
    cv = po.CURVES["bn254"]
    n, log_n = 256, 8
    pts = jac_from_affine(cv, co.gen_bases(1, 9, 10, n))
    om = omega_m(cv, n)
    want = co.serial_ec_fft(1, pts, om, log_n, nthreads=16)
    d = ecgpu.DeviceBuffer.upload(prog, pts)
    ecgpu.ec_fft_dev(prog, "bn254", d, om, log_n)
    assert same_points(1, d.read(shape=pts.shape), want)
