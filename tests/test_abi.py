"""CPU tests of the drop-in boundary: libecgpu.so loads and exports every
symbol include/ecgpu.h declares; host-side logic of the API mirror; and the
product path's independence from the oracle.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import ecgpu
from conftest import ROOT, load_npz

HEADER = os.path.join(ROOT, "include", "ecgpu.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ecg_[a-z0-9_]+)\s*\(", text)) - {"ecg_abort_cb"})


def test_library_exports_every_declared_symbol():
    L = ecgpu.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    # and the binding declares a signature for each of them
    assert set(syms) <= set(ecgpu._SIGS), set(syms) - set(ecgpu._SIGS)


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", ecgpu.LIB_PATH],
                         capture_output=True, text=True)
    blob = open(ecgpu.LIB_PATH, "rb").read()
    assert b"gfx950" in blob, "libecgpu.so must embed gfx950 code objects"
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_product_does_not_link_or_import_the_oracle():
    out = subprocess.run(["readelf", "-d", ecgpu.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    src_dir = os.path.join(ROOT, "0g-ec-gpu_amd")
    for dp, _, files in os.walk(src_dir):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp")):
                text = open(os.path.join(dp, f)).read()
                assert "coracle" not in text and "py_oracle" not in text and "liboracle" not in text, f


def test_version_and_error_string():
    assert b"gfx950" in ecgpu.lib().ecg_version()
    assert isinstance(ecgpu.last_error(), str)


def test_check_bases_reproduces_cpu_error():
    g = load_npz("msm_bls12_381.npz")
    B, E = g["bases_3"].copy(), g["exps_3"].copy()
    ecgpu.check_bases("bls12_381", B, E)           # fixture: fine
    B[2] = 0                                        # identity base with non-zero scalar
    E[2] = [7, 0, 0, 0]
    with pytest.raises(ecgpu.EcError, match="identity element in the CRS"):
        ecgpu.check_bases("bls12_381", B, E)
    E[2] = 0                                        # zero scalar: allowed
    ecgpu.check_bases("bls12_381", B, E)


def test_no_device_behaviour():
    if ecgpu.lib().ecg_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert ecgpu.Device.all() == []
    with pytest.raises(ecgpu.EcError, match="No working GPUs found!"):
        ecgpu.FftKernel.create([])
    with pytest.raises(ecgpu.EcError, match="No working GPUs found!"):
        ecgpu.MultiexpKernel.create([], [])
    h = ctypes.c_void_p()
    assert ecgpu.lib().ecg_ctx_create(0, ctypes.byref(h)) == ecgpu.ECG_ERR_NODEV
    assert "No working GPUs found!" in ecgpu.last_error()


def test_source_builder_and_generate():
    sb = ecgpu.SourceBuilder.new().add_fft("bls12_381_fr").add_multiexp("bls12_381").add_multiexp("bn254")
    assert sb.fields == {"bls12_381_fr", "bls12_381_fq", "bn254_fr", "bn254_fq"}
    assert "fft bls12_381_fr" in sb.build_32_bit_limbs()
    ecgpu.generate(sb)
    with pytest.raises(ecgpu.EcError):
        ecgpu.generate(ecgpu.SourceBuilder.new().add_fft("bls12_381_fq"))
    ecgpu.generate(ecgpu.SourceBuilder.new().add_ec_fft("bls12_381").add_ec_fft("bn254"))
    with pytest.raises(ecgpu.EcError):
        ecgpu.generate(ecgpu.SourceBuilder.new().add_ec_fft("bls12_377"))


def _limbs(x: int) -> np.ndarray:
    return np.array([(x >> (64 * i)) & (2**64 - 1) for i in range(max(1, (x.bit_length() + 63) // 64))],
                    dtype=np.uint64)


def test_kernel_registry_from_moduli():
    """ecg_field_id / ecg_curve_id resolve an instantiation from the moduli
    ag_types::GpuField::modulus() reports, as the Rust ag_build / program!
    shims do (integration/rust/ecgpu-sys/src/lib.rs)."""
    import py_oracle as po

    L = ecgpu.lib()
    fr, fq = po.BLS12_381_FR.modulus, po.BLS12_381_FQ.modulus
    bfr, bfq = po.BN254_FR.modulus, po.BN254_FQ.modulus

    def fid(p, degree=1, pad=0):
        m = np.concatenate([_limbs(p), np.zeros(pad, np.uint64)])
        return L.ecg_field_id(m.ctypes.data_as(ecgpu._u64p), len(m), degree)

    assert fid(fr) == ecgpu.FIELD_BLS12_381_FR and fid(fr, pad=2) == ecgpu.FIELD_BLS12_381_FR
    assert fid(fq) == ecgpu.FIELD_BLS12_381_FQ and fid(bfr) == ecgpu.FIELD_BN254_FR and fid(bfq) == ecgpu.FIELD_BN254_FQ
    assert fid(fq, 2) == ecgpu.FIELD_NAMES["bls12_381_fq2"] and fid(bfq, 2) == ecgpu.FIELD_NAMES["bn254_fq2"]
    assert fid(fr + 2) == ecgpu.ECG_ERR_INVALID and "modulus 0x73eda753" in ecgpu.last_error()
    assert fid(fr, 2) == ecgpu.ECG_ERR_INVALID

    def cid(base, degree, scalar):
        b, sc = _limbs(base), _limbs(scalar)
        return L.ecg_curve_id(b.ctypes.data_as(ecgpu._u64p), len(b), degree, sc.ctypes.data_as(ecgpu._u64p), len(sc))

    assert cid(fq, 1, fr) == ecgpu.CURVE_BLS12_381 and cid(bfq, 1, bfr) == ecgpu.CURVE_BN254
    assert cid(fq, 2, fr) == ecgpu.CURVE_BLS12_381_G2 and cid(bfq, 2, bfr) == ecgpu.CURVE_BN254_G2
    assert cid(fq, 1, bfr) == ecgpu.ECG_ERR_INVALID and "no curve" in ecgpu.last_error()

    K = ecgpu
    assert L.ecg_has_kernel(K.KIND_FFT, K.FIELD_BLS12_381_FR) == 1 and L.ecg_has_kernel(K.KIND_FFT, K.FIELD_BN254_FR) == 1
    assert L.ecg_has_kernel(K.KIND_FFT, K.FIELD_BLS12_381_FQ) == 0          # no 2-adic roots in Fq
    for c in range(4):
        for kind in (K.KIND_EC, K.KIND_EC_FFT, K.KIND_MULTIEXP):
            assert L.ecg_has_kernel(kind, c) == 1
    assert L.ecg_has_kernel(K.KIND_MULTIEXP, 7) == 0 and L.ecg_has_kernel(9, 0) == 0
    assert L.ecg_field_name(0) == b"bls12_381_fr" and L.ecg_curve_name(3) == b"bn254_g2"
    assert L.ecg_field_name(17) is None and L.ecg_curve_name(-1) is None


def test_source_builder_g2_fields():
    sb = ecgpu.SourceBuilder.new().add_multiexp("bls12_381_g2").add_ec_fft("bn254_g2")
    assert {"bls12_381_fq2", "bls12_381_fq", "bls12_381_fr", "bn254_fq2", "bn254_fq"} <= sb.fields
    ecgpu.generate(sb)


def test_worker_threads_env(monkeypatch):
    monkeypatch.setenv("EC_GPU_NUM_THREADS", "12")   # threadpool.rs:25-30
    w = ecgpu.Worker()
    assert w.num_threads == 12 and w.log_num_threads() == 3


def test_shard_and_fft_assignment():
    from ecgpu.dist import fft_assignment, shard_range

    # multiexp.rs:332-336 contiguous ceil(n / world) ranges
    assert [shard_range(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert [shard_range(2, 4, r) for r in range(4)] == [(0, 1), (1, 2), (2, 2), (2, 2)]
    assert shard_range(0, 3, 1) == (0, 0)
    n = 1 << 26
    assert sum(b - a for a, b in (shard_range(n, 8, r) for r in range(8))) == n
    # fft.rs:216-225 chunks of ceil(m / #dev)
    assert fft_assignment(3, 2) == [[0, 1], [2]]
    assert fft_assignment(5, 8)[:5] == [[0], [1], [2], [3], [4]]
    assert fft_assignment(0, 2) == [[], []]
