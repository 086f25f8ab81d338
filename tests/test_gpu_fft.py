"""GPU parity tests of the HIP NTT through the C ABI (FftKernel mirror).

Model: ec-gpu-proxy/tests/fft.rs (gpu_fft_consistency, log_d 1..=16;
gpu_fft_many_consistency, 3 transforms per call, log_d 1..=20), compared
bit-exactly against the CPU oracle's serial_fft / parallel_fft and against the
committed golden fixtures.  Full-size (2^24) parity is in bench.py and
test_fft_2p24_matches_parallel_fft below."""
import hashlib
import json
import os

import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po
from conftest import GOLDEN, load_npz

pytestmark = pytest.mark.gpu

FIELDS = [("bls12_381_fr", 0), ("bn254_fr", 2)]


def rand_mont(f, n, seed):
    rng = np.random.default_rng(seed)
    # uniform limbs reduced below r: any value < r is a valid Montgomery form
    a = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64((1 << (f.bits - 192 - 1)) - 1)  # < 2^(bits-1) < r
    return a


@pytest.fixture(scope="module")
def kernels(gpu_programs):
    progs, _ = gpu_programs
    return {name: ecgpu.FftKernel.create(progs, name) for name, _ in FIELDS}


@pytest.mark.parametrize("fname,fid", FIELDS)
def test_fft_golden(kernels, fname, fid):
    g = load_npz(f"fft_{fname}.npz")
    for log_n in range(1, 11):
        a = g[f"in_{log_n}"].copy()
        kernels[fname].radix_fft(a, g[f"omega_{log_n}"], log_n)
        assert (a == g[f"out_{log_n}"]).all(), log_n


def test_config1_fft_2p16_hash(kernels):
    """BASELINE config (1) input run through the GPU path reproduces the
    serial_fft fixture hash."""
    meta = json.load(open(os.path.join(GOLDEN, "fft_bls12_381_fr_2p16.json")))
    f = po.BLS12_381_FR
    n = 1 << 16
    rng = po.Xoshiro256ss(0x0FF70016)
    a = co.u64arr([f.to_mont(rng.field_element(f)) for _ in range(n)], 4)
    assert hashlib.sha256(a.tobytes()).hexdigest() == meta["input_sha256"]
    kernels["bls12_381_fr"].radix_fft(a, co.u64arr([f.to_mont(f.omega(n))], 4)[0], 16)
    assert hashlib.sha256(a.tobytes()).hexdigest() == meta["output_sha256"]


@pytest.mark.parametrize("fname,fid", FIELDS)
def test_gpu_fft_consistency(kernels, fname, fid):
    """tests/fft.rs gpu_fft_consistency: log_d 1..=16 (plus 17..20), GPU == CPU."""
    f = po.FIELDS[fname]
    for log_d in range(1, 21):
        n = 1 << log_d
        a = rand_mont(f, n, 1000 + log_d)
        om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
        ref = co.serial_fft(fid, a, om, log_d) if log_d <= 12 else co.parallel_fft(fid, a, om, log_d, 3)
        g = a.copy()
        kernels[fname].radix_fft_many([g], [om], [log_d])
        assert (g == ref).all(), log_d


def test_gpu_fft_many_consistency(kernels):
    """tests/fft.rs gpu_fft_many_consistency: 3 transforms per call."""
    f = po.BLS12_381_FR
    for log_d in (1, 5, 9, 13, 17):
        n = 1 << log_d
        ins = [rand_mont(f, n, 7 * log_d + j) for j in range(3)]
        om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
        refs = [co.serial_fft(0, a, om, log_d) if log_d <= 12 else co.parallel_fft(0, a, om, log_d, 2) for a in ins]
        outs = [a.copy() for a in ins]
        kernels["bls12_381_fr"].radix_fft_many(outs, [om] * 3, [log_d] * 3)
        for o, r in zip(outs, refs):
            assert (o == r).all(), log_d


def test_fft_many_mixed_sizes_and_omegas(kernels):
    f = po.BLS12_381_FR
    sizes = [3, 11, 8, 14]
    ins = [rand_mont(f, 1 << s, s) for s in sizes]
    oms = [co.u64arr([f.to_mont(pow(f.omega(1 << s), 3, f.modulus))], 4)[0] for s in sizes]  # other generators
    refs = [co.serial_fft(0, a, om, s) for a, om, s in zip(ins, oms, sizes)]
    outs = [a.copy() for a in ins]
    kernels["bls12_381_fr"].radix_fft_many(outs, oms, sizes)
    for o, r in zip(outs, refs):
        assert (o == r).all()


def test_fft_edge_values(kernels):
    f = po.BLS12_381_FR
    n = 1 << 9
    om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
    for vals in ([0] * n, [f.modulus - 1] * n, [1] + [0] * (n - 1)):
        a = co.u64arr([f.to_mont(v) for v in vals], 4)
        ref = co.serial_fft(0, a, om, 9)
        kernels["bls12_381_fr"].radix_fft(a, om, 9)
        assert (a == ref).all()


def test_inverse_round_trip_2p22(kernels):
    """Size-independent property at 2^22: FFT(omega^-1) o FFT(omega) = n * id."""
    f = po.BLS12_381_FR
    log_n = 22
    n = 1 << log_n
    a = rand_mont(f, n, 22)
    w = f.omega(n)
    om = co.u64arr([f.to_mont(w)], 4)[0]
    om_inv = co.u64arr([f.to_mont(pow(w, -1, f.modulus))], 4)[0]
    b = a.copy()
    k = kernels["bls12_381_fr"]
    k.radix_fft(b, om, log_n)
    k.radix_fft(b, om_inv, log_n)
    # compare b == n * a on a sample of rows (exact field arithmetic)
    idx = np.random.default_rng(0).integers(0, n, size=512)
    for i in idx:
        x = f.from_mont(co.to_ints(a[i:i + 1])[0])
        y = f.from_mont(co.to_ints(b[i:i + 1])[0])
        assert y == x * n % f.modulus


@pytest.mark.parametrize("fname,fid", FIELDS)
def test_fft_2p24_matches_parallel_fft(kernels, fname, fid):
    """BASELINE config (2) and config (5)'s Fr NTT: 2^24 on one MI355X,
    bit-exact vs CPU parallel_fft (tests/fft.rs:86-176 runs the production
    path against the CPU at its largest size), for BLS12-381 and BN254 Fr."""
    f = po.FIELDS[fname]
    log_n = 24
    a = rand_mont(f, 1 << log_n, 24 + fid)
    om = co.u64arr([f.to_mont(f.omega(1 << log_n))], 4)[0]
    ref = co.parallel_fft(fid, a, om, log_n, 4)
    kernels[fname].radix_fft(a, om, log_n)
    assert (a == ref).all()


def test_fft_errors_and_abort(kernels, gpu_programs):
    f = po.BLS12_381_FR
    k = kernels["bls12_381_fr"]
    om = co.u64arr([f.to_mont(1)], 4)[0]
    with pytest.raises(ecgpu.EcError, match="log_n"):          # reference panics at log_n = 0
        k.radix_fft(np.zeros((1, 4), np.uint64), om, 0)
    progs, _ = gpu_programs
    small = np.zeros((2, 4), np.uint64)
    rc = ecgpu.lib().ecg_fft(progs[0].handle, ecgpu.FIELD_BN254_FR, ecgpu._ptr(small), ecgpu._ptr(om), 29,
                             ecgpu.ABORT_CB(0), None)
    assert rc == ecgpu.ECG_ERR_INVALID and "two-adicity" in ecgpu.last_error()  # BN254 Fr: 2-adicity 28
    rc = ecgpu.lib().ecg_fft(progs[0].handle, ecgpu.FIELD_BLS12_381_FQ, ecgpu._ptr(small), ecgpu._ptr(om), 1,
                             ecgpu.ABORT_CB(0), None)
    assert rc == ecgpu.ECG_ERR_INVALID
    ka = ecgpu.FftKernel.create_with_abort(progs, lambda: True)
    with pytest.raises(ecgpu.Aborted):
        ka.radix_fft(np.zeros((16, 4), np.uint64), om, 4)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("fname,fid,log_n", [("bls12_381_fr", 0, 26), ("bn254_fr", 2, 28)])
def test_fft_large_matches_parallel_fft(kernels, fname, fid, log_n):
    """Sizes above 2^24 up to BN254's two-adicity (fft.rs:14,80-87 accepts up
    to LOG2_MAX_ELEMENTS): 2^26 BLS12-381 Fr (passes of 9/9/8) and 2^28 BN254
    Fr (10/9/9, the largest transform with full per-pass twiddle tables and
    64-bit element indices past 2^31 bytes), bit-exact vs CPU parallel_fft."""
    f = po.FIELDS[fname]
    a = rand_mont(f, 1 << log_n, 100 + log_n)
    om = co.u64arr([f.to_mont(f.omega(1 << log_n))], 4)[0]
    ref = co.parallel_fft(fid, a, om, log_n, 4)
    kernels[fname].radix_fft(a, om, log_n)
    assert (a == ref).all()


@pytest.mark.timeout(600)
def test_fft_2p29_spots_and_round_trip(kernels):
    """2^29 BLS12-381 Fr: above 2^28 the passes run on the split twiddle
    tables (no full per-pass tables, 32-bit-limb butterflies).  Too large for
    the CPU FFT in a test, so: two outputs against their definition
    X_k = sum_j a_j w^(jk) (oracle poly_eval), and FFT(w^-1) o FFT(w) = n id
    on 512 sampled rows."""
    f = po.BLS12_381_FR
    log_n = 29
    n = 1 << log_n
    a = rand_mont(f, n, 29)
    w = f.omega(n)
    om = co.u64arr([f.to_mont(w)], 4)[0]
    om_inv = co.u64arr([f.to_mont(pow(w, -1, f.modulus))], 4)[0]
    k = kernels["bls12_381_fr"]
    b = a.copy()
    k.radix_fft(b, om, log_n)
    for kk in (1, n // 2 + 12345):
        x = co.u64arr([f.to_mont(pow(w, kk, f.modulus))], 4)[0]
        assert (co.poly_eval(0, a, x) == b[kk]).all(), kk
    k.radix_fft(b, om_inv, log_n)
    for i in np.random.default_rng(1).integers(0, n, size=512):
        x = f.from_mont(co.to_ints(a[i:i + 1])[0])
        y = f.from_mont(co.to_ints(b[i:i + 1])[0])
        assert y == x * n % f.modulus


@pytest.mark.timeout(300)
def test_fft_many_with_2p25_among_small(kernels):
    """radix_fft_many (fft.rs:211-246) with a 2^25 input between small ones of
    other sizes and omegas: every output equals its own CPU FFT."""
    f = po.BLS12_381_FR
    sizes = [10, 25, 3, 12, 10]
    ins = [rand_mont(f, 1 << s, 250 + j) for j, s in enumerate(sizes)]
    oms = [co.u64arr([f.to_mont(pow(f.omega(1 << s), 1 + 2 * j, f.modulus))], 4)[0] for j, s in enumerate(sizes)]
    refs = [co.serial_fft(0, a, om, s) if s <= 12 else co.parallel_fft(0, a, om, s, 4)
            for a, om, s in zip(ins, oms, sizes)]
    outs = [a.copy() for a in ins]
    kernels["bls12_381_fr"].radix_fft_many(outs, oms, sizes)
    for o, r, s in zip(outs, refs, sizes):
        assert (o == r).all(), s


@pytest.mark.timeout(900)
@pytest.mark.parametrize("log_n", [31, 32])
def test_fft_2p31_2p32_sparse_spot_outputs(gpu_programs, log_n):
    """2^31 and 2^32 points (68.7 / 137 GB in, the same out, on one GPU with
    its scratch buffer: the reference's LOG2_MAX_ELEMENTS = 32, fft.rs:14):
    element indices past 2^31 on the split twiddle tables.  The input holds 16
    random non-zeros at random positions, so any output X_k = sum_j a_j w^(jk)
    is cheap to compute exactly; 64 random outputs plus the ends are compared,
    which catches a wrong index or twiddle anywhere in the 4-pass schedule."""
    f = po.BLS12_381_FR
    n = 1 << log_n
    r = f.modulus
    rng = np.random.default_rng(2000 + log_n)
    pos = [int(p) for p in rng.choice(n, 16, replace=False)]
    vals = [f.from_mont(co.to_ints(v[None, :])[0]) for v in rand_mont(f, 16, 2000 + log_n)]
    a = np.zeros((n, 4), dtype=np.uint64)
    a[pos] = co.u64arr([f.to_mont(v) for v in vals], 4)
    w = f.omega(n)
    gpu_programs[0][0].release_workspace()  # data + scratch take 275 GB of the 288: hand back the shared scratch
    prog = ecgpu.program(gpu_programs[1][0])  # its own context: 137 GB of workspace, released below
    try:
        ecgpu.FftKernel.create([prog], "bls12_381_fr").radix_fft(a, co.u64arr([f.to_mont(w)], 4)[0], log_n)
    finally:
        prog.close()
    ks = [0, 1, n // 2, n - 1] + [int(k) for k in rng.integers(0, n, 64)]
    for k in ks:
        want = sum(v * pow(w, p * k % n, r) for p, v in zip(pos, vals)) % r
        assert f.from_mont(co.to_ints(a[k:k + 1])[0]) == want, k
