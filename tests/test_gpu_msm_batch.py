"""GPU parity tests of the batched multi-line MSM (ecg_multiple_multiexp), the
path 0g-storage's AMT proofs drive through ag_cuda_ec::multiexp::
multiple_multiexp (ag-cuda-ec/src/multiexp.rs:21-81).

Model: test_multiexp_batch (multiexp.rs:90-146): CHUNK_SIZE 64, CHUNK_NUM 32,
LINES 2, every window size 1..=9, result[line * chunks + chunk] ==
msm_bigint(bases.chunks(64)[k], exps.chunks(64).cycle()[k]).  The reference
compares with arkworks' msm_bigint, which is absent here; the checker is the
oracle's multiexp_cpu restatement (pinned by tests/golden/msm_*.npz), and at
larger sizes the known answer of P_i = (a + i b) G."""
import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po

pytestmark = pytest.mark.gpu

CURVES = [("bls12_381", 0), ("bn254", 1)]
R = {name: po.CURVES[name].fr.modulus for name, _ in CURVES}


def rand_scalars(cv, n, seed):
    rng = po.Xoshiro256ss(seed)
    return co.u64arr([rng.field_element(cv.fr) for _ in range(n)], 4)


def affine_rows(cid, jacs):
    return [co.jac_to_affine(cid, j) for j in jacs]


def expected_tasks(cid, bases, exps, lines, chunks):
    """CPU restatement of the task split (multiexp.cl:228-244): line l, chunk c
    -> sum_i exps[c*clen + i] * bases[l*L + c*clen + i]."""
    L = exps.shape[0]
    clen = L // chunks
    out = []
    for l in range(lines):
        for c in range(chunks):
            b = bases[l * L + c * clen: l * L + (c + 1) * clen]
            e = exps[c * clen: (c + 1) * clen]
            out.append(co.jac_to_affine(cid, co.multiexp_cpu(cid, b, e)) if clen else None)
    return out


def assert_same(cid, got, want):
    assert len(got) == len(want)
    for k, (g, w) in enumerate(zip(affine_rows(cid, got), want)):
        if w is None:
            assert g is None, k
        else:
            assert g is not None and (g == w).all(), k


@pytest.fixture(scope="module")
def prog(gpu_programs):
    return gpu_programs[0][0]


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_batch(prog, cname, cid):
    """multiexp.rs:90-146 shape; every pinned window 1..9 plus the automatic one."""
    cv = po.CURVES[cname]
    CHUNK_SIZE, CHUNK_NUM, LINES = 64, 32, 2
    L = CHUNK_SIZE * CHUNK_NUM
    bases = co.gen_bases(cid, 77, 1009, L * LINES)
    exps = rand_scalars(cv, L, 4242 + cid)
    want = expected_tasks(cid, bases, exps, LINES, CHUNK_NUM)
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    for ws in range(1, 10):
        for neg in (True, False):
            got = ecgpu.multiple_multiexp(prog, d_b, exps, CHUNK_NUM, ws, neg, curve=cname, pin_window=True)
            assert got.shape == (LINES * CHUNK_NUM, 3 * cv.fq.limbs64)
            assert_same(cid, got, want)
    got = ecgpu.multiple_multiexp(prog, d_b, exps, CHUNK_NUM, 8, True, curve=cname)
    assert_same(cid, got, want)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_batch_cycled_amt_shape(prog, cname, cid):
    """benches/amt.rs input style (random_input_by_cycle, periods 97 / 73) at a
    reduced size: 4 lines of 2^13, 2^4 .. 2^7 chunks."""
    cv = po.CURVES[cname]
    LINES, L = 4, 1 << 13
    meta_b = co.gen_bases(cid, 3, 5, 97)
    bases = np.ascontiguousarray(np.resize(meta_b, (L * LINES, meta_b.shape[1])))
    meta_e = rand_scalars(cv, 73, 97 + cid)
    exps = np.ascontiguousarray(np.resize(meta_e, (L, 4)))
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    for chunks in (16, 128):
        want = expected_tasks(cid, bases, exps, LINES, chunks)
        got = ecgpu.multiple_multiexp(prog, d_b, exps, chunks, 6, True, curve=cname)
        assert_same(cid, got, want)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_batch_edges(prog, cname, cid):
    cv = po.CURVES[cname]
    lq = cv.fq.limbs64
    L = 1000
    bases = co.gen_bases(cid, 11, 13, 2 * L)
    exps = rand_scalars(cv, L, 5)
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    # chunk_len = line_len / num_chunks, the remainder ignored (multiexp.cl:230)
    got = ecgpu.multiple_multiexp(prog, d_b, exps, 3, 5, True, curve=cname)
    assert_same(cid, got, expected_tasks(cid, bases, exps, 2, 3))
    # more chunks than terms: every task is the identity (0, 1, 0)
    got = ecgpu.multiple_multiexp(prog, d_b, exps, 2 * L, 5, True, curve=cname)
    one = cv.fq.to_mont(1)
    for row in got:
        assert co.to_ints(row.reshape(3, lq)) == [0, one, 0]
    # one chunk per line == one ordinary MSM per line
    got = ecgpu.multiple_multiexp(prog, d_b, exps, 1, 0, True, curve=cname)
    assert_same(cid, got, expected_tasks(cid, bases, exps, 2, 1))
    # zero, one, r-1 scalars and identity bases (GpuRepr zeros contribute nothing)
    e2 = exps.copy()
    e2[0] = 0
    e2[1] = co.u64arr([1], 4)[0]
    e2[2] = co.u64arr([R[cname] - 1], 4)[0]
    b2 = bases.copy()
    b2[3] = 0
    b2[L + 7] = 0
    d_b2 = ecgpu.upload_multiexp_bases(prog, b2)
    e_ref = e2.copy()
    got = ecgpu.multiple_multiexp(prog, d_b2, e2, 4, 7, True, curve=cname, pin_window=True)
    want = []
    clen = L // 4
    for l in range(2):
        for c in range(4):
            b = b2[l * L + c * clen: l * L + (c + 1) * clen].copy()
            e = e_ref[c * clen: (c + 1) * clen].copy()
            zero_rows = ~b.any(axis=1)
            e[zero_rows] = 0  # identity bases: the oracle needs them out of the sum
            b[zero_rows] = bases[0]
            want.append(co.jac_to_affine(cid, co.multiexp_cpu(cid, b, e)))
    assert_same(cid, got, want)
    # device-resident scalar row
    d_e = ecgpu.DeviceBuffer.upload(prog, exps)
    got = ecgpu.multiple_multiexp(prog, d_b, (d_e, L), 8, 0, True, curve=cname)
    assert_same(cid, got, expected_tasks(cid, bases, exps, 2, 8))


def test_multiexp_batch_errors(prog):
    cv = po.CURVES["bls12_381"]
    bases = co.gen_bases(0, 1, 2, 64)
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    exps = rand_scalars(cv, 64, 1)
    with pytest.raises(ecgpu.EcError):
        ecgpu.multiple_multiexp(prog, d_b, exps, 0)
    with pytest.raises(ecgpu.EcError):
        ecgpu.multiple_multiexp(prog, d_b, exps, 4, 23, pin_window=True)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_batch_kat_large(prog, cname, cid):
    """Known answer for 8 lines x 2^18 with 64 chunks (512 tasks of 4096 terms):
    task (l, c) = (sum_i s_i (a' + i b)) G with a' = a + (l L + c clen) b."""
    cv = po.CURVES[cname]
    LINES, L, CH = 8, 1 << 18, 64
    clen = L // CH
    a, b = 0x1234567, 0x89ABCDEF
    d_b = ecgpu.gen_bases_dev(prog, cname, a, b, LINES * L)
    rng = np.random.default_rng(31337 + cid)
    E = rng.integers(0, 2**64, size=(L, 4), dtype=np.uint64)
    E[:, 3] &= np.uint64((1 << (cv.fr.bits - 192 - 1)) - 1)
    got = ecgpu.multiple_multiexp(prog, d_b, E, CH, 0, True, curve=cname)
    r = R[cname]
    for t in list(range(0, LINES * CH, 37)) + [LINES * CH - 1]:
        l, c = divmod(t, CH)
        a2 = (a + (l * L + c * clen) * b) % r
        k = co.kat_scalar(cid, a2, b, E[c * clen:(c + 1) * clen])
        w = co.jac_to_affine(cid, co.gen_mul(cid, k))
        g = co.jac_to_affine(cid, got[t])
        assert (g is None and w is None) or (g == w).all(), t


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_reference_bench_shape(prog, cname, cid):
    """ag-cuda-ec/benches/multiexp.rs:15-62 as written: 2^22 bases cycled with
    period 99, scalars cycled with period 73 (random_input_by_cycle),
    multiple_multiexp_st(bases, exps, 1024, 8, false) -> 1024 tasks of 4096
    terms, whose sum the bench compares with arkworks.  Here: sampled tasks
    against multiexp_cpu and the sum of all 1024 tasks against the known answer
    (sum_i s_(i mod 73) (a + (i mod 99) b)) G."""
    cv = po.CURVES[cname]
    N, CH = 1 << 22, 1024
    clen = N // CH
    a, b = 41, 43
    meta_b = co.gen_bases(cid, a, b, 99)
    bases = np.ascontiguousarray(np.resize(meta_b, (N, meta_b.shape[1])))
    meta_e = rand_scalars(cv, 73, 73 + cid)
    exps = np.ascontiguousarray(np.resize(meta_e, (N, 4)))
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    got = ecgpu.multiple_multiexp(prog, d_b, exps, CH, 8, False, curve=cname)
    assert got.shape[0] == CH
    for t in (0, 1, 517, CH - 1):
        sl = slice(t * clen, (t + 1) * clen)
        w = co.jac_to_affine(cid, co.multiexp_cpu(cid, bases[sl], exps[sl]))
        g = co.jac_to_affine(cid, got[t])
        assert g is not None and (g == w).all(), t
    i = np.arange(N, dtype=np.int64)
    cnt = np.bincount(i % 73, minlength=73)
    m = np.zeros(73, dtype=np.int64)
    np.add.at(m, i % 73, i % 99)
    r = R[cname]
    k = sum(s * (a * int(cnt[j]) + b * int(m[j])) for j, s in enumerate(co.to_ints(meta_e))) % r
    pts = np.stack([co.jac_to_affine(cid, p) for p in got])
    total = co.naive_multiexp(cid, pts, co.u64arr([1] * CH, 4))
    assert (co.jac_to_affine(cid, total) == co.jac_to_affine(cid, co.gen_mul(cid, k))).all()


@pytest.mark.parametrize("cname,cid", CURVES)
def test_multiexp_batch_many_tasks(prog, cname, cid):
    """More tasks than the host normalises in one batch inversion (> 2048:
    3 lines x 1024 chunks of 8 terms), so the device's per-task normalisation
    runs; every 97th task and the last against multiexp_cpu, plus an identity
    task (all-zero scalars in one chunk)."""
    cv = po.CURVES[cname]
    LINES, L, CH = 3, 1 << 13, 1024
    clen = L // CH
    bases = co.gen_bases(cid, 5, 7, LINES * L)
    exps = rand_scalars(cv, L, 99 + cid)
    exps[3 * clen:4 * clen] = 0
    d_b = ecgpu.upload_multiexp_bases(prog, bases)
    got = ecgpu.multiple_multiexp(prog, d_b, exps, CH, 0, True, curve=cname)
    assert got.shape[0] == LINES * CH
    for t in list(range(0, LINES * CH, 97)) + [3, CH + 3, LINES * CH - 1]:
        l, c = divmod(t, CH)
        b = bases[l * L + c * clen: l * L + (c + 1) * clen]
        e = exps[c * clen: (c + 1) * clen]
        w = co.jac_to_affine(cid, co.multiexp_cpu(cid, b, e))
        g = co.jac_to_affine(cid, got[t])
        assert (g is None and w is None) or (g is not None and w is not None and (g == w).all()), t
