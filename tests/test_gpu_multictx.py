"""GPU tests of the in-process multi-device API with several contexts on the
one GPU of the box (rows a1/a8/a9 of SURVEY §8):

* MultiexpKernel over 3 contexts: parallel_multiexp's ceil(n / #dev) ranges,
  one host thread per context, host fold of the partials
  (ec-gpu-proxy/src/multiexp.rs:324-367,394-397), against multiexp_cpu;
* a context listed twice (its calls serialise on the context lock);
* FftKernel::radix_fft_many / EcFftKernel::radix_ec_fft_many over 3 contexts
  (fft.rs:211-246, ec_fft.rs:224-270) against serial_fft / serial_ec_fft;
* first-writer-wins errors: an abort callback that fires once another worker
  is already running ends the whole call with EcError::Aborted;
* memory-derived MSM passes (calc_chunk_size, multiexp.rs:71-93) and the
  multi-pass loop with its per-pass abort poll (:140-144, :348-361), forced
  to small passes through ecg_ctx_set_msm_chunk."""
import threading

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


def rand_mont(f, n, seed):
    """n values < 2^(bits-1) < r: valid Montgomery forms."""
    a = np.random.default_rng(seed).integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64((1 << (f.bits - 192 - 1)) - 1)
    return a


def same(cid, a, b):
    x, y = co.jac_to_affine(cid, a), co.jac_to_affine(cid, b)
    return (x is None and y is None) or (x is not None and y is not None and (x == y).all())


@pytest.fixture(scope="module")
def progs():
    devs = ecgpu.Device.all()
    assert devs, "no MI355X visible"
    ps = [ecgpu.program(devs[0]) for _ in range(3)]
    yield ps
    for p in ps:
        p.close()


class CountingAbort:
    """maybe_abort that returns True from its k-th call on (thread-safe)."""

    def __init__(self, k):
        self.k, self.calls = k, 0
        self.lock = threading.Lock()

    def __call__(self):
        with self.lock:
            self.calls += 1
            return self.calls >= self.k


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_three_contexts(progs, cname, cid):
    cv = po.CURVES[cname]
    n = (1 << 14) + 5  # ragged: the last context gets a shorter range
    B = co.gen_bases(cid, 300 + cid, 17, n, 8)
    E = rand_scalars(cv, n, 90 + cid)
    want = co.multiexp_cpu(cid, B, E, nthreads=16)
    k = ecgpu.MultiexpKernel.create(progs, [], cname)
    assert k.num_kernels() == 3
    assert same(cid, k.multiexp(ecgpu.Worker(), B, E, 0), want)
    # skip into the bases, as MultiexpKernel::multiexp(bases, exps, skip)
    Bs = np.ascontiguousarray(np.concatenate([co.gen_bases(cid, 5, 5, 7, 2), B]))
    assert same(cid, k.multiexp(ecgpu.Worker(), Bs, E, 7), want)
    # fewer terms than contexts: empty ranges are skipped
    assert same(cid, k.multiexp(ecgpu.Worker(), B[:2], E[:2], 0), co.multiexp_cpu(cid, B[:2], E[:2]))


def test_multiexp_duplicate_context(progs):
    cid, cv = 0, po.BLS12_381
    n = 9000
    B = co.gen_bases(cid, 61, 62, n, 8)
    E = rand_scalars(cv, n, 63)
    k = ecgpu.MultiexpKernel.create([progs[0], progs[0], progs[1]], [], "bls12_381")
    assert same(cid, k.multiexp(ecgpu.Worker(), B, E, 0), co.multiexp_cpu(cid, B, E, nthreads=16))


def test_multiexp_abort_first_writer_wins(progs):
    """The callback fires on its 2nd poll: one worker aborts, the call returns
    Aborted (the other workers' results are discarded)."""
    cid, cv = 0, po.BLS12_381
    n = 6000
    B = co.gen_bases(cid, 71, 72, n, 8)
    E = rand_scalars(cv, n, 73)
    k = ecgpu.MultiexpKernel.create_with_abort(progs, [], CountingAbort(2), "bls12_381")
    with pytest.raises(ecgpu.Aborted):
        k.multiexp(ecgpu.Worker(), B, E, 0)
    # the contexts stay usable after the abort
    k2 = ecgpu.MultiexpKernel.create(progs, [], "bls12_381")
    assert same(cid, k2.multiexp(ecgpu.Worker(), B, E, 0), co.multiexp_cpu(cid, B, E, nthreads=16))


def fr_input(f, n, seed):
    rng = po.Xoshiro256ss(seed)
    return co.u64arr([f.to_mont(rng.field_element(f)) for _ in range(n)], 4)


@pytest.mark.parametrize("fname,fid", [("bls12_381_fr", 0), ("bn254_fr", 2)])
def test_fft_many_three_contexts(progs, fname, fid):
    f = po.BLS12_381_FR if fid == 0 else po.BN254_FR
    log_ns = [10, 3, 12, 7, 11]  # 5 transforms over 3 contexts: chunks of 2
    ins = [fr_input(f, 1 << ln, 500 + i) for i, ln in enumerate(log_ns)]
    oms = [co.u64arr([f.to_mont(f.omega(1 << ln))], 4)[0] for ln in log_ns]
    want = [co.serial_fft(fid, a, om, ln) for a, om, ln in zip(ins, oms, log_ns)]
    ecgpu.FftKernel.create(progs, fname).radix_fft_many(ins, oms, log_ns)
    for a, w in zip(ins, want):
        assert (a == w).all()


@pytest.mark.parametrize("fname,fid", [("bls12_381_fr", 0), ("bn254_fr", 2)])
def test_fft_many_batched_runs(progs, fname, fid):
    """Runs of same-size, same-omega inputs go through one batched transform
    per context (ecgpu.cpp fft_batch: every pass launches the whole run's
    tiles): runs of 1-8 inputs at 2^9-2^16 (one- and two-pass plans), a
    different omega inside a run of one size, and a 2^20 pair, each input
    against the CPU restatement."""
    f = po.BLS12_381_FR if fid == 0 else po.BN254_FR
    log_ns = [16] * 8 + [9] * 3 + [14, 14] + [16] * 2 + [20, 20] + [13] + [1] * 3 + [2] * 2
    oms = [co.u64arr([f.to_mont(f.omega(1 << ln))], 4)[0] for ln in log_ns]
    oms[12] = co.u64arr([f.to_mont(pow(f.omega(1 << 14), -1, f.modulus))], 4)[0]  # inverse omega inside the 2^14 run
    ins = [fr_input(f, 1 << ln, 900 + i) if ln <= 16 else
           np.random.default_rng(900 + i).integers(0, 2**62, size=(1 << ln, 4), dtype=np.uint64)
           for i, ln in enumerate(log_ns)]
    want = [co.parallel_fft(fid, a, om, ln, 3) if ln >= 3 else co.serial_fft(fid, a, om, ln)
            for a, om, ln in zip(ins, oms, log_ns)]
    ecgpu.FftKernel.create(progs[:1], fname).radix_fft_many(ins, oms, log_ns)
    for i, (a, w) in enumerate(zip(ins, want)):
        assert (a == w).all(), i


def test_fft_many_abort(progs):
    f = po.BLS12_381_FR
    log_ns = [12] * 6
    ins = [fr_input(f, 1 << ln, 700 + i) for i, ln in enumerate(log_ns)]
    oms = [co.u64arr([f.to_mont(f.omega(1 << ln))], 4)[0] for ln in log_ns]
    k = ecgpu.FftKernel.create_with_abort(progs, CountingAbort(3), "bls12_381_fr")
    with pytest.raises(ecgpu.Aborted):
        k.radix_fft_many(ins, oms, log_ns)


def test_ec_fft_many_three_contexts(progs):
    cid = 0
    f = po.BLS12_381_FR
    lq = 6
    one = co.u64arr([po.BLS12_381.fq.to_mont(1)], lq)[0]
    log_ns = [4, 6, 5, 3]
    ins, oms = [], []
    for i, ln in enumerate(log_ns):
        aff = co.gen_bases(cid, 31 + i, 7, 1 << ln, 4)
        ins.append(np.ascontiguousarray(np.concatenate([aff, np.tile(one, (1 << ln, 1))], axis=1)))
        oms.append(co.u64arr([f.to_mont(f.omega(1 << ln))], 4)[0])
    want = [co.serial_ec_fft(cid, a.copy(), om, ln) for a, om, ln in zip(ins, oms, log_ns)]
    ecgpu.EcFftKernel.create(progs, "bls12_381").radix_ec_fft_many(ins, oms, log_ns)
    for a, w in zip(ins, want):
        for p, q in zip(a, w):
            assert same(cid, p, q)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_ec_fft_many_batched_runs(progs, cname, cid):
    """Runs of same-size, same-omega EC-FFT inputs as one batched transform
    (ecgpu.cpp ec_fft_batch: every stage launches the whole run's butterflies,
    two GLV lanes each on BLS12-381): runs of 5 at 2^8, 3 at 2^6 with the
    inverse omega in the middle (the run splits), a single 2^7 and a pair of
    2^9, each against serial_ec_fft."""
    cv = po.CURVES[cname]
    f, lq = cv.fr, cv.fq.limbs64
    one = co.u64arr([cv.fq.to_mont(1)], lq)[0]
    log_ns = [8] * 5 + [6] * 3 + [7] + [9, 9]
    ins, oms = [], []
    for i, ln in enumerate(log_ns):
        aff = co.gen_bases(cid, 77 + i, 13, 1 << ln, 4)
        ins.append(np.ascontiguousarray(np.concatenate([aff, np.tile(one, (1 << ln, 1))], axis=1)))
        w = f.omega(1 << ln)
        oms.append(co.u64arr([f.to_mont(pow(w, -1, f.modulus) if i == 6 else w)], 4)[0])
    want = [co.serial_ec_fft(cid, a.copy(), om, ln) for a, om, ln in zip(ins, oms, log_ns)]
    ecgpu.EcFftKernel.create(progs[:1], cname).radix_ec_fft_many(ins, oms, log_ns)
    for k, (a, w) in enumerate(zip(ins, want)):
        for p, q in zip(a, w):
            assert same(cid, p, q), k


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_pass_size_from_memory(progs, cname, cid):
    """calc_chunk_size analogue: sized from the 288 GB of HBM, a 2^26-term MSM
    is one pass; at most 2^31 - 1 terms per pass."""
    p = progs[0]
    n = p.msm_chunk_size(cname)
    assert (1 << 26) < n <= (1 << 31) - 1
    k = ecgpu.MultiexpKernel.create([p], [], cname)
    assert k.kernels[0].n == n


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_host_pipeline_multi_batch(progs, cname, cid):
    """the pipelined host MSM with more passes than
    bucket slots (ecg_msm -> msm_host_t).  Passes pinned to 2^12 terms: 2^15 + 37 terms are 9 passes,
    i.e. a batch of 8 slots and a batch of 1, each with its own reduction
    (CORE_FIN), the batches folded on the host.  With the context capped at
    300 MB (ecg_ctx_set_mem_limit) no second bucket slot fits the budget
    (msm_slot_cap): 9 batches of one slot.  Both equal multiexp_cpu and the
    resident one-pass MSM."""
    cv = po.CURVES[cname]
    n = (1 << 15) + 37
    B = co.gen_bases(cid, 900 + cid, 5, n, 8)
    E = rand_scalars(cv, n, 910 + cid)
    want = co.multiexp_cpu(cid, B, E, nthreads=16)
    p = progs[1]
    d_b = ecgpu.DeviceBuffer.upload(p, B)
    d_e = ecgpu.DeviceBuffer.upload(p, E)
    assert same(cid, ecgpu.msm_dev(p, cname, d_b, d_e, n), want)
    k = ecgpu.MultiexpKernel.create([p], [], cname)
    p.set_msm_chunk(1 << 12)
    try:
        assert same(cid, k.multiexp(ecgpu.Worker(), B, E, 0), want)
        p.set_mem_limit(300 << 20)
        assert same(cid, k.multiexp(ecgpu.Worker(), B, E, 0), want)
    finally:
        p.set_mem_limit(0)
        p.set_msm_chunk(0)
        d_b.free()
        d_e.free()


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_multi_pass(progs, cname, cid):
    """Passes forced to 2^12 terms: n = 2^14 + 37 runs as 5 passes (window
    sums folded per pass on the host) and must equal multiexp_cpu; an abort
    on the second poll stops the call between passes."""
    cv = po.CURVES[cname]
    n = (1 << 14) + 37
    B = co.gen_bases(cid, 800 + cid, 3, n, 8)
    E = rand_scalars(cv, n, 810 + cid)
    want = co.multiexp_cpu(cid, B, E, nthreads=16)
    p = progs[1]
    p.set_msm_chunk(1 << 12)
    try:
        assert p.msm_chunk_size(cname) == 1 << 12
        k = ecgpu.MultiexpKernel.create([p], [], cname)
        assert same(cid, k.multiexp(ecgpu.Worker(), B, E, 0), want)
        # two pinned contexts: 2 ranges x 3 passes
        progs[2].set_msm_chunk(1 << 12)
        k2 = ecgpu.MultiexpKernel.create([p, progs[2]], [], cname)
        assert same(cid, k2.multiexp(ecgpu.Worker(), B, E, 0), want)
        ab = CountingAbort(2)
        ka = ecgpu.MultiexpKernel.create_with_abort([p], [], ab, cname)
        with pytest.raises(ecgpu.Aborted):
            ka.multiexp(ecgpu.Worker(), B, E, 0)
        assert ab.calls == 2  # polled before pass 1 (continue) and pass 2 (abort)
    finally:
        p.set_msm_chunk(0)
        progs[2].set_msm_chunk(0)
    assert p.msm_chunk_size(cname) > 1 << 26


def test_release_workspace_then_rerun(progs):
    """ecg_ctx_release_workspace frees a context's scratch and its cached
    twiddle tables: the same NTT and MSM afterwards regrow them and return the
    same bytes (the tables are rebuilt, not read from freed memory)."""
    p = progs[0]
    f = po.BLS12_381_FR
    log_n = 16
    a = rand_mont(f, 1 << log_n, 77)
    w = co.u64arr([f.to_mont(f.omega(1 << log_n))], 4)[0]
    fk = ecgpu.FftKernel.create([p], "bls12_381_fr")
    x0 = a.copy()
    fk.radix_fft(x0, w, log_n)
    cv = po.CURVES["bn254"]
    n = 1 << 14
    B = co.gen_bases(1, 31, 7, n, 8)
    E = rand_scalars(cv, n, 32)
    d_b = ecgpu.DeviceBuffer.upload(p, B)
    d_e = ecgpu.DeviceBuffer.upload(p, E)
    m0 = ecgpu.msm_dev(p, "bn254", d_b, d_e, n)
    p.release_workspace()
    p.release_workspace()  # twice: nothing left to free
    x1 = a.copy()
    fk.radix_fft(x1, w, log_n)
    assert (x1 == x0).all()
    assert same(1, ecgpu.msm_dev(p, "bn254", d_b, d_e, n), m0)
    d_b.free()
    d_e.free()

