"""GPU parity tests of ecg_msm_ex, the MSM with the reference's host-side prep
on device: DensityTracker::generate_exps (multiexp_cpu.rs:
127-138) + MultiexpKernel::multiexp(bases, exps, skip), Montgomery exps
(to_bigint, ag-types/src/impls.rs:13), ark Affine {x, y, infinity} bases
(impls.rs:48-58), and the persistent base cache.  Checker: the oracle's
multiexp_cpu on host-prepared inputs."""
import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po

pytestmark = pytest.mark.gpu

CURVES = [("bls12_381", 0), ("bn254", 1)]


def rand_scalars(cv, n, seed):
    rng = po.Xoshiro256ss(seed)
    return co.u64arr([rng.field_element(cv.fr) for _ in range(n)], 4)


def same(cid, a, b):
    x, y = co.jac_to_affine(cid, a), co.jac_to_affine(cid, b)
    return (x is None and y is None) or (x is not None and y is not None and (x == y).all())


@pytest.fixture(scope="module")
def kernels(gpu_programs):
    progs, devs = gpu_programs
    return {name: ecgpu.MultiexpKernel.create(progs, devs, name) for name, _ in CURVES}


@pytest.mark.parametrize("cname,cid", CURVES)
def test_density_skip_montgomery(kernels, cname, cid):
    cv = po.CURVES[cname]
    k = kernels[cname]
    N = 5003  # not a multiple of 64
    rng = np.random.default_rng(10 + cid)
    bits = rng.random(N) < 0.45
    D = int(bits.sum())
    skip = 17
    bases = co.gen_bases(cid, 21, 23, D + skip + 5)
    exps = rand_scalars(cv, N, 99 + cid)
    dens = ecgpu.DensityTracker(bits)
    want = co.multiexp_cpu(cid, bases[skip:skip + D], exps[bits], nthreads=8)
    got = k.multiexp_ex(bases, exps, skip=skip, density=dens)
    assert same(cid, got, want)
    # Montgomery-form exps give the same point
    em = co.to_mont(2 * cid, exps)
    got = k.multiexp_ex(bases, em, skip=skip, density=dens, exps_montgomery=True)
    assert same(cid, got, want)
    # FullDensity == plain multiexp
    got = k.multiexp_ex(bases, exps[:D], skip=skip, density=ecgpu.FullDensity())
    assert same(cid, got, co.multiexp_cpu(cid, bases[skip:skip + D], exps[:D], nthreads=8))
    # empty density -> identity; too few bases -> the reference's error
    got = k.multiexp_ex(bases, exps, density=ecgpu.DensityTracker(np.zeros(N, dtype=bool)))
    assert co.jac_to_affine(cid, got) is None
    with pytest.raises(ecgpu.EcError, match="Expected more bases from source"):
        k.multiexp_ex(bases, exps, skip=skip + 6, density=dens)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_ark_affine_layout_and_cache(kernels, cname, cid):
    cv = po.CURVES[cname]
    lq = cv.fq.limbs64
    k = kernels[cname]
    n = 3000
    bases = co.gen_bases(cid, 5, 6, n)
    exps = rand_scalars(cv, n, 7 + cid)
    ark = np.zeros((n, 2 * lq + 1), dtype=np.uint64)
    ark[:, :2 * lq] = bases
    inf = [4, 100, n - 1]
    ark[inf, 2 * lq] = 1          # infinity flag
    ark[inf, :2 * lq] = 12345     # junk coordinates must be ignored
    ref_b = bases.copy()
    ref_e = exps.copy()
    ref_e[inf] = 0                # identity bases contribute nothing
    want = co.multiexp_cpu(cid, ref_b, ref_e, nthreads=8)
    got = k.multiexp_ex(ark, exps, ark_affine=True)
    assert same(cid, got, want)
    # cached bases: the first call uploads, the second reuses the device copy
    got1 = k.multiexp_ex(ark, exps, ark_affine=True, cache_bases=True)
    got2 = k.multiexp_ex(ark, exps, ark_affine=True, cache_bases=True)
    assert same(cid, got1, want) and same(cid, got2, want)
    # skip into a cached array
    got = k.multiexp_ex(ark, exps[:1000], skip=1500, ark_affine=True, cache_bases=True)
    # (no infinity record falls in [1500, 2500))
    assert same(cid, got, co.multiexp_cpu(cid, bases[1500:2500], exps[:1000], nthreads=8))
    k.clear_base_cache()


def test_multiple_multiexp_montgomery_exps(gpu_programs):
    prog = gpu_programs[0][0]
    cv = po.CURVES["bls12_381"]
    L, chunks = 1024, 8
    bases = co.gen_bases(0, 8, 9, 2 * L)
    exps = rand_scalars(cv, L, 5)
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    a = ecgpu.multiple_multiexp(prog, d_b, exps, chunks)
    b = ecgpu.multiple_multiexp(prog, d_b, co.to_mont(0, exps), chunks, exps_montgomery=True)
    for x, y in zip(a, b):
        assert same(0, x, y)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_base_cache_not_stale(kernels, cname, cid):
    """A cached entry is keyed by the host address; an array with other
    content at the same address (a freed array's memory reused) must not be
    served the old bases: the content fingerprint catches it."""
    cv = po.CURVES[cname]
    k = kernels[cname]
    n = 2048
    buf = co.gen_bases(cid, 41, 42, n)
    exps = rand_scalars(cv, n, 77 + cid)
    got1 = k.multiexp_ex(buf, exps, cache_bases=True)
    assert same(cid, got1, co.multiexp_cpu(cid, buf, exps, nthreads=8))
    buf[:] = co.gen_bases(cid, 43, 44, n)   # same address, every record different
    got2 = k.multiexp_ex(buf, exps, cache_bases=True)
    assert same(cid, got2, co.multiexp_cpu(cid, buf, exps, nthreads=8))
    # a temporary copy cannot be cached by address
    with pytest.raises(ecgpu.EcError, match="cache_bases"):
        k.multiexp_ex(buf.astype(np.int64), exps, cache_bases=True)
    k.clear_base_cache()


@pytest.mark.parametrize("cname,cid", CURVES)
def test_cached_ark_pipelined_2p22(gpu_programs, cname, cid):
    """The Rust drop-in's MultiexpKernel::multiexp path at a size that takes
    the pipelined branch (cached bases, >= 2^22 host exponents): arkworks
    Affine records read on the device, cached as prepared records, then the
    exponents in geometrically growing passes whose buckets share one
    reduction.  With skip, identity bases and Montgomery exponents; checked
    against the resident single-pass MSM and the known answer
    sum s_i (a + (skip + i) b) G."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    prog = gpu_programs[0][0]
    r_int = bench.R_BLS if cid == 0 else bench.R_BN
    lq = ecgpu.CURVE_FQ_LIMBS[cid]
    skip, n = 777, (1 << 22) + 12345
    a, b = 1234567, 89101112
    d_b = ecgpu.gen_bases_dev(prog, cname, a, b, n + skip)
    xy = d_b.read(shape=(n + skip, 2 * lq))
    d_b.free()
    ark = np.zeros((n + skip, 2 * lq + 1), dtype=np.uint64)
    ark[:, :2 * lq] = xy
    ident = [skip + 5, skip + n // 2, skip + n - 1]  # identity bases (infinity set) contribute nothing
    ark[ident, :2 * lq] = 0
    ark[ident, 2 * lq] = 1
    xy[ident] = 0
    E = bench.rand_scalars(np.random.default_rng(cid + 222), n, r_int)
    k = ecgpu.MultiexpKernel.create([prog], [], cname)
    k.clear_base_cache()
    first = k.multiexp_ex(ark, E, skip=skip, ark_affine=True, cache_bases=True)
    again = k.multiexp_ex(ark, co.to_mont(2 * cid, E), skip=skip, ark_affine=True, cache_bases=True,
                          exps_montgomery=True)
    d_xy = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(xy[skip:]))
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    resident = ecgpu.msm_dev(prog, cname, d_xy, d_e, n)
    assert (first == resident).all() and (again == resident).all()
    E_kat = E.copy()
    E_kat[[i - skip for i in ident]] = 0  # identity bases: their terms vanish
    kat = co.kat_scalar(cid, (a + skip * b) % r_int, b, E_kat, nthreads=16) % r_int
    assert (co.jac_to_affine(cid, first) == co.jac_to_affine(cid, co.gen_mul(cid, kat))).all()
    # cold fill (skip 0, every base used): the cache entry is built pass by pass
    # inside the pipelined MSM -- ark records and [x, y] records
    for arr, ark_l in ((ark[skip:], True), (np.ascontiguousarray(xy[skip:]), False)):
        k.clear_base_cache()
        cold = k.multiexp_ex(arr, E, 0, ark_affine=ark_l, cache_bases=True)
        hit = k.multiexp_ex(arr, E, 0, ark_affine=ark_l, cache_bases=True)
        assert (cold == resident).all() and (hit == resident).all()
    k.clear_base_cache()
    d_xy.free()
    d_e.free()
