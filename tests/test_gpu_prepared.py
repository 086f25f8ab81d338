"""GPU parity tests of prepared bases (ecg_msm_prepare_bases): the device-side
half of ag-cuda-ec's upload_multiexp_bases (ag-cuda-ec/src/multiexp.rs:11-19)
-- bases converted once into the bucket kernels' layout, then consumed by
msm_dev, multiple_multiexp and the multi-pass MSM.  Checker: multiexp_cpu on
the same bases (and the unprepared device path)."""
import ctypes

import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po

pytestmark = pytest.mark.gpu

CURVES = [("bls12_381", 0), ("bn254", 1), ("bls12_381_g2", 2), ("bn254_g2", 3)]


def rand_scalars(cv, n, seed):
    rng = po.Xoshiro256ss(seed)
    return co.u64arr([rng.field_element(cv.fr) for _ in range(n)], 4)


def same(cid, a, b):
    x, y = co.jac_to_affine(cid, a), co.jac_to_affine(cid, b)
    return (x is None and y is None) or (x is not None and y is not None and (x == y).all())


@pytest.fixture(scope="module")
def prog(gpu_programs):
    return gpu_programs[0][0]


@pytest.mark.parametrize("cname,cid", CURVES[:2])
def test_prepared_msm_dev(prog, cname, cid):
    """Prepared G1 bases (reduced-radix records) give the multiexp_cpu point,
    for the whole array and for a shorter prefix; identity bases included."""
    cv = po.CURVES[cname]
    n = (1 << 16) + 77
    d_b = ecgpu.gen_bases_dev(prog, cname, 31 + cid, 7, n)
    B = d_b.read(shape=(n, -1))
    B[5] = 0  # GpuRepr identity
    d_b.write(B)
    E = rand_scalars(cv, n, 40 + cid)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    pb = ecgpu.prepare_bases(prog, cname, d_b, n)
    want = co.multiexp_cpu(cid, np.delete(B, 5, axis=0), np.delete(E, 5, axis=0), nthreads=16)
    assert same(cid, ecgpu.msm_dev(prog, cname, pb, d_e, n), want)
    assert same(cid, ecgpu.msm_dev(prog, cname, d_b, d_e, n), want)
    m = 1000  # a prefix of the prepared bases (the identity at 5 dropped for the CPU checker)
    want_m = co.multiexp_cpu(cid, np.delete(B[:m], 5, axis=0), np.delete(E[:m], 5, axis=0), nthreads=8)
    assert same(cid, ecgpu.msm_dev(prog, cname, pb, d_e, m), want_m)
    pb.free()
    d_b.free()
    d_e.free()


@pytest.mark.parametrize("cname,cid", CURVES[2:])
def test_prepared_g2(prog, cname, cid):
    """G2 keeps the [x, y] layout: prepared bases are a device copy and give
    the same point as the unprepared path (itself pinned by test_gpu_g2)."""
    n = (1 << 12) + 3
    d_b = ecgpu.gen_bases_dev(prog, cname, 11 + cid, 13, n)
    rng = np.random.default_rng(cid)
    E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    E[:, 3] &= np.uint64(2**60 - 1)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    want = ecgpu.msm_dev(prog, cname, d_b, d_e, n)
    pb = ecgpu.prepare_bases(prog, cname, d_b, n)
    d_b.free()
    # both outputs are normalised Jacobian (x, y, 1) or (0, 1, 0): compare words
    assert (ecgpu.msm_dev(prog, cname, pb, d_e, n) == want).all()
    pb.free()
    d_e.free()


@pytest.mark.parametrize("cname,cid", CURVES[:2])
def test_prepared_multi_pass(prog, cname, cid):
    """Passes forced to 2^12 terms over prepared bases: per-pass record
    offsets in the prepared layout."""
    cv = po.CURVES[cname]
    n = (1 << 14) + 37
    B = co.gen_bases(cid, 900 + cid, 5, n, 8)
    E = rand_scalars(cv, n, 910 + cid)
    want = co.multiexp_cpu(cid, B, E, nthreads=16)
    d_b = ecgpu.DeviceBuffer.upload(prog, B)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    pb = ecgpu.prepare_bases(prog, cname, d_b, n)
    prog.set_msm_chunk(1 << 12)
    try:
        assert same(cid, ecgpu.msm_dev(prog, cname, pb, d_e, n), want)
    finally:
        prog.set_msm_chunk(0)
    pb.free()
    d_b.free()
    d_e.free()


@pytest.mark.parametrize("cname,cid", CURVES[:2])
def test_prepared_multiple_multiexp(prog, cname, cid):
    """upload_multiexp_bases(curve=...) -> PreparedBases feed multiple_multiexp
    (test_multiexp_batch shape: lines x chunks sharing one scalar row)."""
    cv = po.CURVES[cname]
    L, lines, chunks = 1 << 12, 3, 4
    B = co.gen_bases(cid, 70 + cid, 3, L * lines, 8)
    E = rand_scalars(cv, L, 80 + cid)
    raw = ecgpu.upload_multiexp_bases(prog, B)
    want = ecgpu.multiple_multiexp(prog, raw, E, chunks, curve=cname)
    pb = ecgpu.upload_multiexp_bases(prog, B, curve=cname)
    assert isinstance(pb, ecgpu.PreparedBases)
    got = ecgpu.multiple_multiexp(prog, pb, E, chunks, curve=cname)
    c = L // chunks
    for t in range(lines * chunks):
        line, ch = divmod(t, chunks)
        assert same(cid, got[t], want[t])
        if t in (0, lines * chunks - 1):
            ref = co.multiexp_cpu(cid, B[line * L + ch * c:line * L + (ch + 1) * c], E[ch * c:(ch + 1) * c], nthreads=8)
            assert same(cid, got[t], ref)
    pb.free()
    raw.free()


def test_prepared_errors(prog):
    """A prepared buffer serves only its curve and at most its n bases; freed
    buffers are unregistered; PreparedBases cannot be written or read."""
    n = 1 << 12
    d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 3, 5, n)
    E = rand_scalars(po.CURVES["bls12_381"], n + 1, 7)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    pb = ecgpu.prepare_bases(prog, "bls12_381", d_b, n)
    with pytest.raises(ecgpu.EcError, match="prepared bases"):
        ecgpu.msm_dev(prog, "bls12_381", pb, d_e, n + 1)
    with pytest.raises(ecgpu.EcError, match="prepared bases"):
        ecgpu.msm_dev(prog, "bn254", pb, d_e, 16)
    with pytest.raises(ecgpu.EcError):
        pb.write(E)
    with pytest.raises(ecgpu.EcError):
        pb.read()
    pb.free()
    pb.free()  # idempotent
    d_b.free()
    d_e.free()


def test_prepared_registry_across_contexts_and_views(prog):
    """The prepared-bases registry is process-wide and range-keyed: a buffer
    prepared on one context is read as records from another context on the
    same device, base-aligned pointers into it (views) read the bases from
    there, a pointer off a record boundary is refused, and a buffer freed on
    another context is unregistered (the address then reads as raw [x, y])."""
    cid, cname = 0, "bls12_381"
    cv = po.CURVES[cname]
    n = 5000
    B = co.gen_bases(cid, 61, 67, n, 8)
    E = rand_scalars(cv, n, 71)
    other = ecgpu.program(prog.device)  # a second context on the same GPU
    d_b = ecgpu.DeviceBuffer.upload(prog, B)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    pb = ecgpu.prepare_bases(prog, cname, d_b, n)
    want = co.multiexp_cpu(cid, B, E, nthreads=8)
    assert same(cid, ecgpu.msm_dev(other, cname, pb, d_e, n), want)
    # a view of bases [1000, 1000 + 3000) in the prepared form
    v = pb.view(1000, 3000)
    d_e2 = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(E[1000:4000]))
    assert same(cid, ecgpu.msm_dev(other, cname, v, d_e2, 3000),
                co.multiexp_cpu(cid, B[1000:4000], E[1000:4000], nthreads=8))
    with pytest.raises(ecgpu.EcError, match="prepared bases"):  # from base 1000 the buffer holds n - 1000
        ecgpu.msm_dev(prog, cname, pb.view(1000), d_e, n - 999)
    odd = ecgpu.PreparedBases(prog, ctypes.c_void_p(pb.ptr.value + 64), cid, 10)
    with pytest.raises(ecgpu.EcError, match="base boundary"):
        ecgpu.msm_dev(prog, cname, odd, d_e, 10)
    odd.ptr = None
    assert pb.stride() == 128
    # free through the other context: unregistered with its memory
    ecgpu.lib().ecg_dev_free(other.handle, pb.ptr)
    pb.ptr = None
    # a prepared buffer released behind the library's back (hipFree of its
    # allocation) and the address reused by raw [x, y] bases: the header nonce
    # no longer matches, so the address reads as raw bases again
    pb2 = ecgpu.prepare_bases(prog, cname, d_b, n)
    hip = ctypes.CDLL(ecgpu.lib().ecg_runtime_info().decode().split("(")[1].split(")")[0])
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hdr = 256  # msm.hip PREP_HEADER
    ptr = pb2.ptr.value
    prog.synchronize()
    assert hip.hipFree(ctypes.c_void_p(ptr - hdr)) == 0
    pb2.ptr = None
    d_raw = ecgpu.DeviceBuffer(prog, n * 128 + hdr)
    d_raw.write(np.concatenate([np.zeros(hdr // 8, np.uint64), B.reshape(-1)]))
    if d_raw.ptr.value + hdr == ptr:  # the allocator handed the address back
        raw_view = ecgpu.PreparedBases(prog, ctypes.c_void_p(ptr), cid, n)
        out = np.zeros(18, np.uint64)
        ecgpu._check(ecgpu.lib().ecg_msm_dev(prog.handle, cid, raw_view.ptr, d_e.ptr, n,
                                             out.ctypes.data_as(ctypes.c_void_p), 0, None))
        raw_view.ptr = None
        assert same(cid, out, want)
    d_raw.free()
    # deterministic form of the reuse (the allocator may not hand the address
    # back): a live prepared allocation whose header and records another owner
    # overwrote with raw [x, y] bases.  The header is checked on the stream
    # (msm.hip prep_check_kernel); the mismatch is found after the call, the
    # entry dropped and the call redone over the raw bases -- same result
    pb4 = ecgpu.prepare_bases(prog, cname, d_b, n)
    ptr4 = pb4.ptr.value
    prog.synchronize()
    raw = np.ascontiguousarray(np.concatenate([np.zeros(hdr // 8, np.uint64), B.reshape(-1)]))
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(ctypes.c_void_p(ptr4 - hdr), raw.ctypes.data_as(ctypes.c_void_p), raw.nbytes, 1) == 0
    view4 = ecgpu.PreparedBases(prog, ctypes.c_void_p(ptr4), cid, n)
    for _ in range(2):  # the second call finds no entry: a plain raw-bases MSM
        out = np.zeros(18, np.uint64)
        ecgpu._check(ecgpu.lib().ecg_msm_dev(prog.handle, cid, view4.ptr, d_e.ptr, n,
                                             out.ctypes.data_as(ctypes.c_void_p), 0, None))
        assert same(cid, out, want)
    view4.ptr = None
    assert hip.hipFree(ctypes.c_void_p(ptr4 - hdr)) == 0
    pb4.ptr = None
    # the same, with a reused allocation that starts AT the old records address
    # (the old header address is then outside it, or unmapped): the lookup must
    # not read the header there, and the address reads as raw bases
    pb3 = ecgpu.prepare_bases(prog, cname, d_b, n)
    ptr3 = pb3.ptr.value
    prog.synchronize()
    assert hip.hipFree(ctypes.c_void_p(ptr3 - hdr)) == 0
    pb3.ptr = None
    held = []
    for size in (n * 96, n * 128 + hdr, n * 96 + 4096):
        d = ecgpu.DeviceBuffer(prog, size)
        held.append(d)
        if d.ptr.value == ptr3:
            d.write(B)
            out = np.zeros(18, np.uint64)
            ecgpu._check(ecgpu.lib().ecg_msm_dev(prog.handle, cid, d.ptr, d_e.ptr, n,
                                                 out.ctypes.data_as(ctypes.c_void_p), 0, None))
            assert same(cid, out, want)
            break
    for d in held:
        d.free()
    for buf in (d_b, d_e, d_e2):
        buf.free()
    other.close()


def test_stale_entry_refused_call_confirms_header(prog):
    """a call that the registry would refuse -- more bases than a
    prepared entry holds, or a window-table entry in the grid split -- first
    checks the entry's header on the stream.  When another owner has
    overwritten the allocation with raw [x, y] bases, the entry is dropped and
    the call runs over the raw bases (same result as multiexp_cpu) instead of
    being refused now and at every later call."""
    cid, cname = 0, "bls12_381"
    cv = po.CURVES[cname]
    n = 3000
    hdr = 256  # msm.hip PREP_HEADER
    hip = ctypes.CDLL(ecgpu.lib().ecg_runtime_info().decode().split("(")[1].split(")")[0])
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    m = n * 4 // 3  # raw [x, y] bases (96 B) that fit in n prepared 128-B records
    B = co.gen_bases(cid, 71, 73, m, 8)
    E = rand_scalars(cv, m, 75)
    d_b = ecgpu.DeviceBuffer.upload(prog, B[:n])
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    raw = np.ascontiguousarray(np.concatenate([np.zeros(hdr // 8, np.uint64), B.reshape(-1)]))

    def overwrite(pb):
        prog.synchronize()
        assert hip.hipMemcpy(ctypes.c_void_p(pb.ptr.value - hdr), raw.ctypes.data_as(ctypes.c_void_p), raw.nbytes, 1) == 0
        return ecgpu.PreparedBases(prog, ctypes.c_void_p(pb.ptr.value), cid, m)

    try:
        # a plain prepared entry of n records, read as m > n raw bases
        pb = ecgpu.prepare_bases(prog, cname, d_b, n)
        view = overwrite(pb)
        want = co.multiexp_cpu(cid, B, E, nthreads=8)
        for _ in range(2):  # the second call finds no entry
            out = np.zeros(18, np.uint64)
            ecgpu._check(ecgpu.lib().ecg_msm_dev(prog.handle, cid, view.ptr, d_e.ptr, m,
                                                 out.ctypes.data_as(ctypes.c_void_p), 0, None))
            assert same(cid, out, want)
        view.ptr = None
        assert hip.hipFree(ctypes.c_void_p(pb.ptr.value - hdr)) == 0
        pb.ptr = None
        # a window-table entry in the grid split (which refuses tables): its allocation holds the
        # table's W rows per base, plenty for the raw bases
        tb = ecgpu.prepare_bases(prog, cname, d_b, n, window_table=8)
        view = overwrite(tb)
        part, _ = ecgpu.msm_grid_part(prog, cname, view, d_e, n, 0, 1)
        assert same(cid, part, co.multiexp_cpu(cid, B[:n], E[:n], nthreads=8))
        view.ptr = None
        assert hip.hipFree(ctypes.c_void_p(tb.ptr.value - hdr)) == 0
        tb.ptr = None
    finally:
        d_b.free()
        d_e.free()
