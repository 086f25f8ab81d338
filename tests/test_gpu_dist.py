"""GPU tests of the multi-GPU path that a single-GPU box can run.

* ecg_fft_dist's schedule (all-to-all, stage1 T-point DFT + twiddle,
  all-to-all, local NTT, all-to-all, stage3 interleave) with T = 2, 4, 8
  block buffers on one GPU and the exchanges done by host copies
  (ecgpu.dist.fft_dist_emulated): every device kernel of the distributed NTT
  runs, and the result must equal the CPU serial_fft (fft_cpu.rs:10-52) of
  the whole array, bit-exact.
* the RCCL communicator itself at world size 1 (ecg_comm_init /
  ecg_msm_dist / ecg_fft_dist): id creation, init, exchange-as-copy.
Multi-rank RCCL needs one GPU per rank; it runs in the driver's 8-GPU
bench (bench.py --gpus N)."""
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
