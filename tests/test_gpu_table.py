"""GPU parity tests of window tables (ecg_msm_prepare_table): fixed bases
prepared once with their 2^(k c) multiples, so every window of an MSM feeds
one bucket set.  The bases-reused-across-MSMs use of upload_multiexp_bases
(ag-cuda-ec/src/multiexp.rs:11-19).  Checker: multiexp_cpu on the same bases
(multiexp_cpu.rs:244-367 restated in oracle/oracle.c) and the other base
forms of the same engine."""
import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po

pytestmark = pytest.mark.gpu

G1 = [("bls12_381", 0), ("bn254", 1)]


def rand_scalars(cv, n, seed):
    rng = po.Xoshiro256ss(seed)
    return co.u64arr([rng.field_element(cv.fr) for _ in range(n)], 4)


def same(cid, a, b):
    x, y = co.jac_to_affine(cid, a), co.jac_to_affine(cid, b)
    return (x is None and y is None) or (x is not None and y is not None and (x == y).all())


@pytest.fixture(scope="module")
def prog(gpu_programs):
    return gpu_programs[0][0]


@pytest.mark.parametrize("window", [0, 5, 13, 21])
@pytest.mark.parametrize("cname,cid", G1)
def test_table_msm(prog, cname, cid, window):
    """Window tables of several window sizes (auto, small, mid, larger than
    the per-window plan would take) give the multiexp_cpu point, for the whole
    array and a prefix; an identity base included."""
    cv = po.CURVES[cname]
    n = (1 << 15) + 77
    d_b = ecgpu.gen_bases_dev(prog, cname, 131 + cid, 17, n)
    B = d_b.read(shape=(n, -1))
    B[9] = 0  # GpuRepr identity
    d_b.write(B)
    E = rand_scalars(cv, n, 140 + cid + window)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    tab = ecgpu.prepare_bases(prog, cname, d_b, n, window_table=window)
    want = co.multiexp_cpu(cid, np.delete(B, 9, axis=0), np.delete(E, 9, axis=0), nthreads=16)
    assert same(cid, ecgpu.msm_dev(prog, cname, tab, d_e, n), want)
    m = 3001
    want_m = co.multiexp_cpu(cid, np.delete(B[:m], 9, axis=0), np.delete(E[:m], 9, axis=0), nthreads=8)
    assert same(cid, ecgpu.msm_dev(prog, cname, tab, d_e, m), want_m)
    tab.free()
    d_b.free()
    d_e.free()


@pytest.mark.parametrize("cname,cid", G1)
def test_table_edge_scalars(prog, cname, cid):
    """Scalars 0, 1, r-1, 2^256-1 (reduced mod r on device), all-equal digits
    (one heavy bucket shared by every window) and a top-window carry: the
    table path equals the plain prepared path."""
    cv = po.CURVES[cname]
    n = 1 << 14
    d_b = ecgpu.gen_bases_dev(prog, cname, 7 + cid, 3, n)
    r = cv.fr.modulus
    vals = [0, 1, r - 1, 2**256 - 1, (1 << 254) + 12345, 2**24 - 1]
    E = co.u64arr([vals[i % len(vals)] if i < 600 else (2**24 - 1) * (1 + 2**24 + 2**48) for i in range(n)], 4)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    plain = ecgpu.prepare_bases(prog, cname, d_b, n)
    tab = ecgpu.prepare_bases(prog, cname, d_b, n, window_table=24)
    assert same(cid, ecgpu.msm_dev(prog, cname, tab, d_e, n), ecgpu.msm_dev(prog, cname, plain, d_e, n))
    tab.free()
    plain.free()
    d_b.free()
    d_e.free()


@pytest.mark.parametrize("cname,cid", G1)
def test_table_multi_pass(prog, cname, cid):
    """Passes forced to 2^12 terms over a window table: the per-pass base
    offset inside each table row."""
    cv = po.CURVES[cname]
    n = (1 << 14) + 37
    B = co.gen_bases(cid, 950 + cid, 5, n, 8)
    E = rand_scalars(cv, n, 960 + cid)
    want = co.multiexp_cpu(cid, B, E, nthreads=16)
    d_b = ecgpu.DeviceBuffer.upload(prog, B)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    tab = ecgpu.prepare_bases(prog, cname, d_b, n, window_table=11)
    prog.set_msm_chunk(1 << 12)
    try:
        assert same(cid, ecgpu.msm_dev(prog, cname, tab, d_e, n), want)
    finally:
        prog.set_msm_chunk(0)
    tab.free()
    d_b.free()
    d_e.free()


@pytest.mark.parametrize("window", [8, 12])
@pytest.mark.parametrize("cname,cid", G1)
def test_table_multiple_multiexp(prog, cname, cid, window):
    """multiple_multiexp over a window table (lines x chunks sharing one
    scalar row, the AMT shape in small): equal to the untabled batched MSM
    task by task, two tasks also against multiexp_cpu."""
    cv = po.CURVES[cname]
    L, lines, chunks = 1 << 12, 3, 8
    B = co.gen_bases(cid, 170 + cid, 3, L * lines, 8)
    E = rand_scalars(cv, L, 180 + cid + window)
    raw = ecgpu.upload_multiexp_bases(prog, B)
    want = ecgpu.multiple_multiexp(prog, raw, E, chunks, curve=cname)
    tab = ecgpu.upload_multiexp_bases(prog, B, curve=cname, window_table=window)
    got = ecgpu.multiple_multiexp(prog, tab, E, chunks, curve=cname)
    c = L // chunks
    for t in range(lines * chunks):
        assert same(cid, got[t], want[t]), t
    for t in (0, lines * chunks - 1):
        line, ch = divmod(t, chunks)
        ref = co.multiexp_cpu(cid, B[line * L + ch * c:line * L + (ch + 1) * c], E[ch * c:(ch + 1) * c], nthreads=8)
        assert same(cid, got[t], ref)
    tab.free()
    raw.free()


def test_table_errors(prog):
    """G2 has no table form; window sizes outside [2, 25] and tables past the
    2^31 index space are refused; a table serves at most its n bases."""
    n = 1 << 10
    d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 3, 5, n)
    with pytest.raises(ecgpu.EcError, match="G1"):
        g2 = ecgpu.gen_bases_dev(prog, "bls12_381_g2", 3, 5, 16)
        try:
            ecgpu.prepare_bases(prog, "bls12_381_g2", g2, 16, window_table=8)
        finally:
            g2.free()
    for c in (1, 26):
        with pytest.raises(ecgpu.EcError, match="window size"):
            ecgpu.prepare_bases(prog, "bls12_381", d_b, n, window_table=c)
    with pytest.raises(ecgpu.EcError, match="2\\^31"):
        ecgpu.prepare_bases(prog, "bls12_381", d_b, 1 << 28, window_table=4)
    tab = ecgpu.prepare_bases(prog, "bls12_381", d_b, n, window_table=9)
    E = rand_scalars(po.CURVES["bls12_381"], n + 1, 7)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    with pytest.raises(ecgpu.EcError, match="prepared bases"):
        ecgpu.msm_dev(prog, "bls12_381", tab, d_e, n + 1)
    tab.free()
    d_b.free()
    d_e.free()
