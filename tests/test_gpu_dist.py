"""GPU tests of the multi-GPU path that a single-GPU box can run.

* ecg_fft_dist's schedule (all-to-all, stage1 T-point DFT + twiddle,
  all-to-all, local NTT, all-to-all, stage3 interleave) with T = 2, 4, 8
  block buffers on one GPU and the exchanges done by host copies
  (ecgpu.dist.fft_dist_emulated): every device kernel of the distributed NTT
  runs, and the result must equal the CPU serial_fft (fft_cpu.rs:10-52) of
  the whole array, bit-exact.
* the RCCL communicator itself at world size 1 (ecg_comm_init /
  ecg_msm_dist / ecg_fft_dist): id creation, init, exchange-as-copy, and a
  real one-rank RCCL communicator (non-blocking init, the status records,
  the deadline-bounded waits).
* ecg_msm_dist / ecg_fft_dist at world 2-8 with one context per rank on the
  one GPU and the host transport (ecg_comm_init_host, threads): the same C
  code path as the RCCL ranks -- shard, status exchange, payload exchange,
  fold -- only the bytes move through host memory.  This covers BASELINE
  config 4 at its real per-rank size (8 x 2^23 shards of one prepared 2^26
  base set, c = 16 / W = 16 / one sort) with the 2^26 known answer, and the
  multi-rank failure semantics (a failing or aborting rank makes every rank
  return the same error; multiexp.rs:345-365, fft.rs:218-245).
Multi-rank RCCL needs one GPU per rank; it runs in the driver's 8-GPU
bench (bench.py --gpus N)."""
import ctypes
import os
import sys
import threading
import time

import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po
from ecgpu import dist as edist

pytestmark = pytest.mark.gpu

FIELDS = [("bls12_381_fr", 0), ("bn254_fr", 2)]


def rand_fr(f, n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64((1 << (f.bits - 192 - 1)) - 1)  # < r, any value is a Montgomery form
    return a


@pytest.mark.parametrize("fname,fid", FIELDS)
@pytest.mark.parametrize("T", [2, 4, 8])
def test_fft_dist_emulated(gpu_programs, fname, fid, T):
    f = po.FIELDS[fname]
    prog = gpu_programs[0][0]
    progs = [prog] * T
    for log_n in (7, 12, 16):
        if (1 << log_n) < 2 * T * T:
            continue
        n = 1 << log_n
        a = rand_fr(f, n, 1000 * T + log_n)
        om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
        want = co.serial_fft(fid, a.copy(), om, log_n)
        m = n // T
        blocks = [ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(a[r * m:(r + 1) * m])) for r in range(T)]
        edist.fft_dist_emulated(progs, fname, blocks, om, log_n)
        got = np.concatenate([b.read(shape=(m, 4)) for b in blocks])
        assert (got == want).all(), (T, log_n)


def test_comm_world1(gpu_programs):
    prog = gpu_programs[0][0]
    edist.comm_init(prog, 0, 1)
    # ecg_fft_dist at world 1 == the plain NTT
    f = po.FIELDS["bls12_381_fr"]
    log_n = 14
    n = 1 << log_n
    a = rand_fr(f, n, 77)
    om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
    d = ecgpu.DeviceBuffer.upload(prog, a)
    edist.fft_dist(prog, "bls12_381_fr", d, om, log_n)
    assert (d.read(shape=(n, 4)) == co.serial_fft(0, a.copy(), om, log_n)).all()
    # ecg_msm_dist at world 1 == the MSM
    cv = po.CURVES["bls12_381"]
    nb = 4096
    bases = co.gen_bases(0, 3, 4, nb)
    rng = po.Xoshiro256ss(5)
    e = co.u64arr([rng.field_element(cv.fr) for _ in range(nb)], 4)
    d_b = ecgpu.DeviceBuffer.upload(prog, bases)
    d_e = ecgpu.DeviceBuffer.upload(prog, e)
    got = edist.msm_dist(prog, "bls12_381", d_b, d_e, nb)
    want = co.multiexp_cpu(0, bases, e, nthreads=8)
    assert (co.jac_to_affine(0, got) == co.jac_to_affine(0, want)).all()
    # the RCCL id itself (librccl loads, ncclGetUniqueId works)
    import ctypes
    buf = (ctypes.c_uint8 * 128)()
    ecgpu._check(ecgpu.lib().ecg_comm_unique_id(buf))
    ecgpu.lib().ecg_comm_destroy(prog.handle)


def test_fft_dist_rejects_bad_shapes(gpu_programs):
    prog = gpu_programs[0][0]
    lib = ecgpu.lib()
    d = ecgpu.DeviceBuffer(prog, 1 << 12)
    om = np.zeros(4, dtype=np.uint64)
    with pytest.raises(ecgpu.EcError):  # 3 ranks: not a power of two
        ecgpu._check(lib.ecg_fft_dist_stage1(prog.handle, 0, d.ptr, d.ptr, ecgpu._ptr(om), 3, 0, 10))
    with pytest.raises(ecgpu.EcError):  # 2^4 points over 4 ranks: m/T < 1
        ecgpu._check(lib.ecg_fft_dist_stage1(prog.handle, 0, d.ptr, d.ptr, ecgpu._ptr(om), 4, 0, 4))
    with pytest.raises(ecgpu.EcError):  # rank out of range
        ecgpu._check(lib.ecg_fft_dist_stage1(prog.handle, 0, d.ptr, d.ptr, ecgpu._ptr(om), 2, 2, 10))


def test_comm_world1_rccl(gpu_programs):
    """A real one-rank RCCL communicator: non-blocking init under a deadline,
    the [status | partial] all-gather, both status exchanges of the
    distributed NTT, a failing call answered on the rank, the communicator
    still usable after it."""
    prog = ecgpu.program(gpu_programs[1][0])
    try:
        edist.comm_init(prog, 0, 1, rccl_at_world1=True, timeout_s=120)
        f = po.FIELDS["bn254_fr"]
        log_n = 12
        n = 1 << log_n
        a = rand_fr(f, n, 78)
        om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
        d = ecgpu.DeviceBuffer.upload(prog, a)
        edist.fft_dist(prog, "bn254_fr", d, om, log_n)
        assert (d.read(shape=(n, 4)) == co.serial_fft(2, a.copy(), om, log_n)).all()
        nb = 3000
        bases = co.gen_bases(1, 5, 6, nb)
        e = rand_fr(po.BN254_FR, nb, 6)
        d_b = ecgpu.DeviceBuffer.upload(prog, bases)
        d_e = ecgpu.DeviceBuffer.upload(prog, e)
        # the first MSM on this context: a workspace failure of its local step
        # (capped by ecg_ctx_set_mem_limit) still runs the status exchange,
        # whose staging was reserved at ecg_comm_init
        prog.set_mem_limit(1 << 12)
        with pytest.raises(ecgpu.EcError, match="ecg_ctx_set_mem_limit"):
            edist.msm_dist(prog, "bn254", d_b, d_e, nb)
        prog.set_mem_limit(0)
        with pytest.raises(ecgpu.EcError, match="unknown curve"):
            edist.msm_dist(prog, 7, d_b, d_e, nb)
        with pytest.raises(ecgpu.Aborted):
            edist.msm_dist(prog, "bn254", d_b, d_e, nb, maybe_abort=lambda: True)
        got = edist.msm_dist(prog, "bn254", d_b, d_e, nb)
        assert (co.jac_to_affine(1, got) == co.jac_to_affine(1, co.multiexp_cpu(1, bases, e, nthreads=8))).all()
        # what the communicator itself reports (bench.py's `rccl` record at N > 1)
        info = edist.comm_info(prog)
        assert info["transport"] == "rccl" and info["count"] == 1 and info["rank"] == 0
        assert info["device"] == gpu_programs[1][0].index and ":" in info["pci_bus_id"]
        assert edist.last_exchange_us(prog) > 0
        for buf in (d, d_b, d_e):
            buf.free()
    finally:
        ecgpu.lib().ecg_comm_destroy(prog.handle)
        prog.close()


def _run_ranks(world, fn, timeout=600):
    """fn(rank) on `world` threads; returns [(ok, value-or-exception)] per rank."""
    out = [None] * world

    def body(r):
        try:
            out[r] = (True, fn(r))
        except BaseException as exc:  # noqa: BLE001 -- reported per rank
            out[r] = (False, exc)

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a rank is still blocked: the failure was not propagated"
    return out


def _host_ranks(dev, world, timeout_s=60):
    ex = edist.LocalExchange(world, timeout_s=timeout_s)
    progs = [ecgpu.program(dev) for _ in range(world)]
    for r, p in enumerate(progs):
        edist.comm_init_host(p, r, world, ex.exchange_for(r), timeout_s=timeout_s)
    return progs


class _Ptr:
    """A device pointer into a larger buffer (a rank's shard view)."""

    def __init__(self, buf, offset):
        self.ptr = ctypes.c_void_p(buf.ptr.value + offset)


@pytest.mark.parametrize("cname,cid", [("bls12_381", 0), ("bn254", 1)])
@pytest.mark.parametrize("world", [2, 4])
def test_msm_fft_dist_host_transport(gpu_programs, cname, cid, world):
    """ecg_msm_dist and ecg_fft_dist with `world` ranks on one GPU: every rank
    returns multiexp_cpu / serial_fft of the whole input, bit-exact."""
    dev = gpu_programs[1][0]
    progs = _host_ranks(dev, world)
    try:
        cv = po.CURVES[cname]
        n = 5003  # ragged: the last shard is shorter
        B = co.gen_bases(cid, 17, 19, n, 8)
        rng = np.random.default_rng(world)
        E = rand_fr(cv.fr, n, world + 10 + cid)
        want = co.multiexp_cpu(cid, B, E, nthreads=8)
        shards = [edist.shard_range(n, world, r) for r in range(world)]
        d_b = [ecgpu.DeviceBuffer.upload(progs[r], np.ascontiguousarray(B[i0:i1]) if i1 > i0 else B[:1])
               for r, (i0, i1) in enumerate(shards)]
        d_e = [ecgpu.DeviceBuffer.upload(progs[r], np.ascontiguousarray(E[i0:i1]) if i1 > i0 else E[:1])
               for r, (i0, i1) in enumerate(shards)]
        res = _run_ranks(world, lambda r: edist.msm_dist(progs[r], cname, d_b[r], d_e[r], shards[r][1] - shards[r][0]))
        for ok, got in res:
            assert ok, got
            assert (co.jac_to_affine(cid, got) == co.jac_to_affine(cid, want)).all()
        # one NTT block-distributed over the ranks
        fname, fid = ("bls12_381_fr", 0) if cid == 0 else ("bn254_fr", 2)
        f = po.FIELDS[fname]
        log_n = 13
        m = (1 << log_n) // world
        a = rand_fr(f, 1 << log_n, int(rng.integers(1 << 30)))
        om = co.u64arr([f.to_mont(f.omega(1 << log_n))], 4)[0]
        ref = co.serial_fft(fid, a.copy(), om, log_n)
        blocks = [ecgpu.DeviceBuffer.upload(progs[r], np.ascontiguousarray(a[r * m:(r + 1) * m])) for r in range(world)]
        res = _run_ranks(world, lambda r: edist.fft_dist(progs[r], fname, blocks[r], om, log_n))
        assert all(ok for ok, _ in res), res
        got = np.concatenate([b.read(shape=(m, 4)) for b in blocks])
        assert (got == ref).all()
        for b in d_b + d_e + blocks:
            b.free()
    finally:
        for p in progs:
            p.close()


def test_dist_failure_semantics(gpu_programs):
    """A failing or aborting rank makes EVERY rank return an error (none is
    left inside an exchange): the lowest failing rank's code on every rank,
    its own message on it and 'rank k failed' on the others; ranks called with
    different arguments are refused; the ranks stay usable afterwards."""
    world = 3
    dev = gpu_programs[1][0]
    progs = _host_ranks(dev, world)
    try:
        cid, cname = 0, "bls12_381"
        n = 999
        B = co.gen_bases(cid, 23, 29, n, 8)
        E = rand_fr(po.BLS12_381_FR, n, 5)
        d_b = [ecgpu.DeviceBuffer.upload(p, B) for p in progs]
        d_e = [ecgpu.DeviceBuffer.upload(p, E) for p in progs]

        def msm(curves, aborts=(False,) * world):
            return _run_ranks(world, lambda r: edist.msm_dist(progs[r], curves[r], d_b[r], d_e[r], n,
                                                              maybe_abort=(lambda: True) if aborts[r] else None))

        # rank 1 passes an unknown curve: all three fail with ECG_ERR_INVALID
        res = msm([cname, 9, cname])
        assert not any(ok for ok, _ in res)
        assert "unknown curve" in str(res[1][1])
        assert "rank 1 of 3 failed" in str(res[0][1]) and "rank 1 of 3 failed" in str(res[2][1])
        # rank 2 aborts (maybe_abort): every rank returns Aborted
        res = msm([cname] * 3, aborts=(False, False, True))
        assert all(isinstance(e, ecgpu.Aborted) for _, e in res), res
        # two failures: the lowest failing rank's code wins everywhere (rank 0 aborted, rank 2 invalid)
        res = msm([cname, cname, 9], aborts=(True, False, False))
        assert all(isinstance(e, ecgpu.Aborted) for _, e in res), res
        # ranks that disagree on the curve (both valid) are refused
        d_b1 = ecgpu.DeviceBuffer.upload(progs[1], co.gen_bases(1, 23, 29, n, 8))
        res = _run_ranks(world, lambda r: edist.msm_dist(progs[r], "bn254" if r == 1 else cname,
                                                         d_b1 if r == 1 else d_b[r], d_e[r], n))
        assert not any(ok for ok, _ in res) and all("curve" in str(e) for _, e in res), res
        d_b1.free()
        # still usable: 3 x the same terms = 3 x the MSM
        res = msm([cname] * 3)
        want = co.multiexp_cpu(cid, np.concatenate([B] * 3), np.concatenate([E] * 3), nthreads=8)
        assert all(ok and (co.jac_to_affine(cid, v) == co.jac_to_affine(cid, want)).all() for ok, v in res), res
        # distributed NTT (world must be a power of two: 3 ranks is refused on every rank)
        f = po.BLS12_381_FR
        om = co.u64arr([f.to_mont(f.omega(1 << 10))], 4)[0]
        blk = [ecgpu.DeviceBuffer(p, (1 << 10) * 32) for p in progs]
        res = _run_ranks(world, lambda r: edist.fft_dist(progs[r], "bls12_381_fr", blk[r], om, 10))
        assert not any(ok for ok, _ in res)
        for b in d_b + d_e + blk:
            b.free()
    finally:
        for p in progs:
            p.close()


def test_dist_workspace_failure_fails_fast(gpu_programs):
    """a rank whose local MSM fails on a workspace
    allocation (here: rank 1 of 3 capped by ecg_ctx_set_mem_limit) still joins
    the status exchange -- the status records need no allocation after the
    local step -- so all three ranks return ECG_ERR_NOMEM within seconds, not
    at the exchange deadline.  comm_info reports the host transport; the same
    ranks then run a good call exactly."""
    world = 3
    dev = gpu_programs[1][0]
    progs = _host_ranks(dev, world, timeout_s=45)
    try:
        cid, cname = 0, "bls12_381"
        n = 5000
        B = co.gen_bases(cid, 31, 37, n, 8)
        E = rand_fr(po.BLS12_381_FR, n, 17)
        d_b = [ecgpu.DeviceBuffer.upload(p, B) for p in progs]
        d_e = [ecgpu.DeviceBuffer.upload(p, E) for p in progs]
        infos = [edist.comm_info(p) for p in progs]
        assert [i["rank"] for i in infos] == [0, 1, 2] and all(i["count"] == 3 for i in infos)
        assert all(i["transport"] == "host" for i in infos)
        rec = edist.comm_record(infos)
        assert rec["distinct"] is False and rec["ranks"] == [0, 1, 2]  # three ranks on one GPU
        progs[1].set_mem_limit(1 << 12)
        t0 = time.perf_counter()
        res = _run_ranks(world, lambda r: edist.msm_dist(progs[r], cname, d_b[r], d_e[r], n), timeout=120)
        elapsed = time.perf_counter() - t0
        assert not any(ok for ok, _ in res), res
        assert all(f"rc={ecgpu.ECG_ERR_NOMEM}" in str(e) for _, e in res), res
        assert "ecg_ctx_set_mem_limit" in str(res[1][1])
        assert "rank 1 of 3 failed" in str(res[0][1]) and "rank 1 of 3 failed" in str(res[2][1])
        assert elapsed < 15, elapsed
        progs[1].set_mem_limit(0)
        res = _run_ranks(world, lambda r: edist.msm_dist(progs[r], cname, d_b[r], d_e[r], n))
        want = co.jac_to_affine(cid, co.multiexp_cpu(cid, np.concatenate([B] * 3), np.concatenate([E] * 3),
                                                     nthreads=8))
        assert all(ok and (co.jac_to_affine(cid, v) == want).all() for ok, v in res), res
        for b in d_b + d_e:
            b.free()
    finally:
        for p in progs:
            p.close()


def test_fft_dist_failure_semantics(gpu_programs):
    """ecg_fft_dist: a bad argument on one rank, an abort before the first
    exchange and an abort after the local NTT (the second status exchange)
    all end the call on every rank; then a good call is exact."""
    world = 2
    dev = gpu_programs[1][0]
    progs = _host_ranks(dev, world)
    try:
        f = po.BLS12_381_FR
        log_n = 11
        m = (1 << log_n) // world
        a = rand_fr(f, 1 << log_n, 99)
        om = co.u64arr([f.to_mont(f.omega(1 << log_n))], 4)[0]
        blocks = [ecgpu.DeviceBuffer.upload(progs[r], np.ascontiguousarray(a[r * m:(r + 1) * m])) for r in range(world)]
        # rank 1 names a field without an NTT
        res = _run_ranks(world, lambda r: edist.fft_dist(progs[r], 1 if r else "bls12_381_fr", blocks[r], om, log_n))
        assert not any(ok for ok, _ in res) and "rank 1 of 2 failed" in str(res[0][1]), res
        # ranks disagree on the size
        res = _run_ranks(world, lambda r: edist.fft_dist(progs[r], "bls12_381_fr", blocks[r], om, log_n - r))
        assert not any(ok for ok, _ in res), res
        # rank 0 aborts at the second poll (after its local NTT): rank 1 stops too
        polls = [0]

        def late_abort():
            polls[0] += 1
            return polls[0] >= 2

        res = _run_ranks(world, lambda r: edist.fft_dist(progs[r], "bls12_381_fr", blocks[r], om, log_n,
                                                         maybe_abort=late_abort if r == 0 else None))
        assert polls[0] == 2 and all(isinstance(e, ecgpu.Aborted) for _, e in res), res
        for r in range(world):
            blocks[r].write(np.ascontiguousarray(a[r * m:(r + 1) * m]))
        res = _run_ranks(world, lambda r: edist.fft_dist(progs[r], "bls12_381_fr", blocks[r], om, log_n))
        assert all(ok for ok, _ in res), res
        got = np.concatenate([b.read(shape=(m, 4)) for b in blocks])
        assert (got == co.serial_fft(0, a.copy(), om, log_n)).all()
        for b in blocks:
            b.free()
    finally:
        for p in progs:
            p.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cname,cid", [("bls12_381", 0), ("bn254", 1)])
def test_config4_msm_2p26_eight_shards(gpu_programs, cname, cid):
    """BASELINE config 4 on one GPU: 2^26 bases generated and prepared ONCE;
    8 ranks (one context each, host transport) each run ecg_msm_dist on their
    2^23 shard -- a base-aligned view into the prepared buffer and the exact
    scalars bench.py gives that rank at N = 8 -- with the per-rank plan
    asserted (c = 16, W = 16, one sort over all window blocks); every rank
    must return the same point, equal to the 2^26 known answer."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    world, n_total = 8, 1 << 26
    r_int = bench.R_BLS if cid == 0 else bench.R_BN
    c, W, mode = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
    ecgpu._check(ecgpu.lib().ecg_msm_plan_info(cid, n_total // world, 0, ctypes.byref(c), ctypes.byref(W),
                                               ctypes.byref(mode)))
    assert (c.value, W.value, mode.value) == (16, 16, 1)  # ECG_SORT_PW_ONE
    prog0 = gpu_programs[0][0]
    d_raw = ecgpu.gen_bases_dev(prog0, cname, bench.KAT_A % r_int, bench.KAT_B, n_total)
    prep = ecgpu.prepare_bases(prog0, cname, d_raw, n_total)
    d_raw.free()
    shards = [bench.msm_shard(r, world, n_total, r_int) for r in range(world)]
    d_sc = ecgpu.DeviceBuffer.upload(prog0, np.concatenate([s[2] for s in shards]))
    progs = _host_ranks(gpu_programs[1][0], world, timeout_s=300)
    try:
        views = [prep.view(i0, n_loc) for i0, n_loc, _, _ in shards]
        res = _run_ranks(world, lambda r: edist.msm_dist(progs[r], cname, views[r], _Ptr(d_sc, shards[r][0] * 32),
                                                         shards[r][1]))
        assert all(ok for ok, _ in res), res
        first = res[0][1]
        assert all((v == first).all() for _, v in res)
        kat = bench.msm_kat_scalar(co, cid, world, n_total, r_int, 16, shards)
        want = co.jac_to_affine(cid, co.gen_mul(cid, kat))
        assert (co.jac_to_affine(cid, first) == want).all()
    finally:
        for p in progs:
            p.close()
        prep.free()
        d_sc.free()


def _fold_parts(cid, parts):
    nq = ecgpu.CURVE_FQ_LIMBS[cid]
    acc = np.zeros(3 * nq, dtype=np.uint64)
    for p in parts:
        p = np.ascontiguousarray(p, dtype=np.uint64)
        co.lib().orc_jac_add(cid, co.ptr(acc), co.ptr(acc), co.ptr(p))
    return acc


@pytest.mark.parametrize("cname,cid", [("bls12_381", 0), ("bn254", 1)])
@pytest.mark.parametrize("prepared", [False, True])
def test_msm_grid_parts(gpu_programs, cname, cid, prepared):
    """Grid split's per-rank step (ecg_msm_grid_part): for rank counts that
    cut windows mid-way (3, 5, 13), exactly on window edges (1, 2, 8) and
    more ranks than grid cells (n = 1), the nranks partials fold to
    multiexp_cpu of the whole input, bit-exact, and no rank runs more than
    three Pippenger pieces (partial window, whole windows, partial window)."""
    prog = gpu_programs[0][0]
    cv = po.CURVES[cname]
    for n, seed in ((5003, 3), (7, 4), (1, 5)):
        B = co.gen_bases(cid, 23, 29, n, 8)
        E = rand_fr(cv.fr, n, seed + 20 * cid)
        want = co.jac_to_affine(cid, co.multiexp_cpu(cid, B, E, nthreads=8))
        d_b = ecgpu.DeviceBuffer.upload(prog, B)
        d_e = ecgpu.DeviceBuffer.upload(prog, E)
        bases = ecgpu.prepare_bases(prog, cname, d_b, n) if prepared else d_b
        try:
            for nranks in (1, 2, 3, 5, 8, 13):
                parts, pieces = [], []
                for r in range(nranks):
                    p, k = ecgpu.msm_grid_part(prog, cname, bases, d_e, n, r, nranks)
                    parts.append(p)
                    pieces.append(k)
                assert max(pieces) <= 3, (n, nranks, pieces)
                got = co.jac_to_affine(cid, _fold_parts(cid, parts))
                assert (got == want).all(), (n, nranks)
        finally:
            if prepared:
                bases.free()
            d_b.free()
            d_e.free()


@pytest.mark.parametrize("cname,cid", [("bls12_381", 0), ("bn254", 1)])
def test_msm_grid_part_chunked_by_pass_budget(gpu_programs, cname, cid):
    """A grid share larger than one device pass (here: the context pinned to
    2^9-term passes, ecg_ctx_set_msm_chunk) runs as several one-call
    sub-ranges whose partials are summed: the ranks' partials
    still fold to multiexp_cpu, and a share reports more than one piece."""
    prog = ecgpu.program(gpu_programs[1][0])
    cv = po.CURVES[cname]
    n = 5003
    B = co.gen_bases(cid, 41, 47, n, 8)
    E = rand_fr(cv.fr, n, 90 + cid)
    want = co.jac_to_affine(cid, co.multiexp_cpu(cid, B, E, nthreads=8))
    d_b = ecgpu.DeviceBuffer.upload(prog, B)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    try:
        prog.set_msm_chunk(1 << 9)
        for nranks in (3, 5):
            parts, pieces = [], []
            for r in range(nranks):
                p, k = ecgpu.msm_grid_part(prog, cname, d_b, d_e, n, r, nranks)
                parts.append(p)
                pieces.append(k)
            assert max(pieces) > 1, pieces
            assert (co.jac_to_affine(cid, _fold_parts(cid, parts)) == want).all(), nranks
    finally:
        d_b.free()
        d_e.free()
        prog.close()


def test_msm_grid_part_rejects(gpu_programs):
    """Bad rank numbers and window-table bases are refused, not run."""
    prog = gpu_programs[0][0]
    n = 64
    B = co.gen_bases(0, 3, 5, n, 2)
    E = rand_fr(po.CURVES["bls12_381"].fr, n, 1)
    d_b = ecgpu.DeviceBuffer.upload(prog, B)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    try:
        for r, nr in ((2, 2), (-1, 2), (0, 0)):
            with pytest.raises(ecgpu.EcError):
                ecgpu.msm_grid_part(prog, "bls12_381", d_b, d_e, n, r, nr)
        tab = ecgpu.prepare_bases(prog, "bls12_381", d_b, n, window_table=8)
        try:
            with pytest.raises(ecgpu.EcError, match="window table"):
                ecgpu.msm_grid_part(prog, "bls12_381", tab, d_e, n, 0, 2)
        finally:
            tab.free()
    finally:
        d_b.free()
        d_e.free()


@pytest.mark.parametrize("cname,cid", [("bls12_381", 0), ("bn254", 1)])
@pytest.mark.parametrize("world", [2, 3])
def test_msm_dist_grid_host_transport(gpu_programs, cname, cid, world):
    """ecg_msm_dist_grid with `world` ranks on one GPU (host transport),
    every rank holding all bases and scalars: every rank returns multiexp_cpu
    of the whole input, bit-exact."""
    progs = _host_ranks(gpu_programs[1][0], world)
    try:
        cv = po.CURVES[cname]
        n = 4099
        B = co.gen_bases(cid, 31, 37, n, 8)
        E = rand_fr(cv.fr, n, 40 + world + cid)
        want = co.jac_to_affine(cid, co.multiexp_cpu(cid, B, E, nthreads=8))
        d_b = [ecgpu.DeviceBuffer.upload(p, B) for p in progs]
        d_e = [ecgpu.DeviceBuffer.upload(p, E) for p in progs]
        res = _run_ranks(world, lambda r: edist.msm_dist_grid(progs[r], cname, d_b[r], d_e[r], n))
        for ok, got in res:
            assert ok, got
            assert (co.jac_to_affine(cid, got) == want).all()
        for b in d_b + d_e:
            b.free()
    finally:
        for p in progs:
            p.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cname,cid", [("bls12_381", 0), ("bn254", 1)])
def test_config4_msm_2p26_grid_split(gpu_programs, cname, cid):
    """BASELINE config 4 through the grid split: 2^26 bases prepared once and
    the 2^26 scalars bench.py generates (all shards concatenated) are shared by
    8 host-transport ranks, each running 1/8 of the (window x term) grid of
    the 2^26 plan; every rank returns the 2^26 known answer."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    world, n_total = 8, 1 << 26
    r_int = bench.R_BLS if cid == 0 else bench.R_BN
    prog0 = gpu_programs[0][0]
    d_raw = ecgpu.gen_bases_dev(prog0, cname, bench.KAT_A % r_int, bench.KAT_B, n_total)
    prep = ecgpu.prepare_bases(prog0, cname, d_raw, n_total)
    d_raw.free()
    shards = [bench.msm_shard(r, world, n_total, r_int) for r in range(world)]
    d_sc = ecgpu.DeviceBuffer.upload(prog0, np.concatenate([s[2] for s in shards]))
    progs = _host_ranks(gpu_programs[1][0], world, timeout_s=300)
    try:
        res = _run_ranks(world, lambda r: edist.msm_dist_grid(progs[r], cname, prep, d_sc, n_total))
        assert all(ok for ok, _ in res), res
        first = res[0][1]
        assert all((v == first).all() for _, v in res)
        kat = bench.msm_kat_scalar(co, cid, world, n_total, r_int, 16, shards)
        want = co.jac_to_affine(cid, co.gen_mul(cid, kat))
        assert (co.jac_to_affine(cid, first) == want).all()
    finally:
        for p in progs:
            p.close()
        prep.free()
        d_sc.free()


def test_msm_dist_grid_failure_semantics(gpu_programs):
    """The grid split shares the range split's status exchange: a rank with an
    unknown curve or an abort makes every rank return the same error, and the
    ranks stay usable (3 ranks, one GPU, host transport)."""
    world = 3
    progs = _host_ranks(gpu_programs[1][0], world)
    try:
        cid, cname = 0, "bls12_381"
        n = 777
        B = co.gen_bases(cid, 5, 7, n, 8)
        E = rand_fr(po.BLS12_381_FR, n, 12)
        d_b = [ecgpu.DeviceBuffer.upload(p, B) for p in progs]
        d_e = [ecgpu.DeviceBuffer.upload(p, E) for p in progs]

        def grid(curves, aborts=(False,) * world):
            return _run_ranks(world, lambda r: edist.msm_dist_grid(
                progs[r], curves[r], d_b[r], d_e[r], n, maybe_abort=(lambda: True) if aborts[r] else None))

        res = grid([cname, 9, cname])
        assert not any(ok for ok, _ in res)
        assert "rank 1 of 3 failed" in str(res[0][1]) and "rank 1 of 3 failed" in str(res[2][1])
        res = grid([cname] * 3, aborts=(False, True, False))
        assert all(isinstance(e, ecgpu.Aborted) for _, e in res), res
        # rank 2 is called with another whole-MSM size: its grid share would not tile
        # the others', so every rank refuses the result (n rides in the record)
        res = _run_ranks(world, lambda r: edist.msm_dist_grid(progs[r], cname, d_b[r], d_e[r], n - 100 if r == 2 else n))
        assert not any(ok for ok, _ in res), res
        assert all("n = " in str(e) for _, e in res), res
        res = grid([cname] * 3)
        want = co.jac_to_affine(cid, co.multiexp_cpu(cid, B, E, nthreads=8))
        assert all(ok and (co.jac_to_affine(cid, v) == want).all() for ok, v in res), res
        for b in d_b + d_e:
            b.free()
    finally:
        for p in progs:
            p.close()
