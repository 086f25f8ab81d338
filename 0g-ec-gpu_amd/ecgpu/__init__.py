"""Host-side mirror of the reference's ec-gpu-gen API over libecgpu.so.

The reference (kriptohaberciniz/0g-ec-gpu) exposes this hot path to Rust
provers as (ec-gpu-proxy/src/{fft,multiexp}.rs, ag-build/src/source/builder.rs,
ec-gpu-program/src/program.rs):

    let sb = ag_build::SourceBuilder::new().add_fft::<Fr>().add_multiexp::<G1Affine>();
    ag_build::generate(&sb);                                   // build.rs
    let programs = Device::all().iter().map(|d| program!(d)).collect()?;
    let mut fft = FftKernel::<Fr>::create(programs)?;
    fft.radix_fft_many(&mut [&mut coeffs], &[omega], &[log_n])?;
    let mut msm = MultiexpKernel::<G1Affine>::create(programs, &devices)?;
    let acc: G1Projective = msm.multiexp(&pool, bases, exps, skip)?;

This module keeps those names, argument meanings and error behaviour, with
numpy uint64 arrays in the arkworks in-memory layouts (see include/ecgpu.h):
Fr elements (n, 4) Montgomery; bases (n, 2*Lq) [x|y] Montgomery (GpuRepr,
identity = zeros); exps (n, 4) canonical BigInt<4>; results (3*Lq,) Jacobian.
There is no CPU fallback: if libecgpu.so is missing this import fails.
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# ECGPU_LIB selects another in-tree build of the same library (A/B of build flags)
LIB_PATH = os.environ.get("ECGPU_LIB") or os.path.join(os.path.dirname(_PKG), "lib", "libecgpu.so")

# ids shared with include/ecgpu.h
FIELD_BLS12_381_FR, FIELD_BLS12_381_FQ, FIELD_BN254_FR, FIELD_BN254_FQ = 0, 1, 2, 3
CURVE_BLS12_381, CURVE_BN254, CURVE_BLS12_381_G2, CURVE_BN254_G2 = 0, 1, 2, 3
FIELD_NAMES = {"bls12_381_fr": 0, "bls12_381_fq": 1, "bn254_fr": 2, "bn254_fq": 3,
               "bls12_381_fq2": 4, "bn254_fq2": 5}  # the Fq2 ids are registry-only (add_field)
CURVE_NAMES = {"bls12_381": 0, "bn254": 1, "bls12_381_g2": 2, "bn254_g2": 3}
# u64 words per point coordinate (Fq for G1, Fq2 = [c0, c1] for G2)
CURVE_FQ_LIMBS = {0: 6, 1: 4, 2: 12, 3: 8}
CURVE_FR_FIELD = {0: FIELD_BLS12_381_FR, 1: FIELD_BN254_FR, 2: FIELD_BLS12_381_FR, 3: FIELD_BN254_FR}
FR_TWO_ADICITY = {FIELD_BLS12_381_FR: 32, FIELD_BN254_FR: 28}

ECG_OK, ECG_ABORTED = 0, 1
ECG_ERR_INVALID, ECG_ERR_HIP, ECG_ERR_NOMEM, ECG_ERR_NODEV, ECG_ERR_RCCL = -1, -2, -3, -4, -5

_u64p = ctypes.POINTER(ctypes.c_uint64)
ABORT_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
# ecg_xchg_cb(op, send, recv, bytes, user): the host transport of ecg_comm_init_host
XCHG_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                           ctypes.c_void_p)
XCHG_ALLGATHER, XCHG_ALLTOALL = 0, 1

# ---------------------------------------------------------------------------
# errors (ec-gpu-program/src/lib.rs:10-32)
# ---------------------------------------------------------------------------


class EcError(Exception):
    """EcError::Simple / GpuTools / Io."""


class Aborted(EcError):
    """EcError::Aborted -- the maybe_abort callback returned true."""


# ---------------------------------------------------------------------------
# library loading (fails loudly: no CPU fallback on the product path)
# ---------------------------------------------------------------------------

_lib = None
_lib_lock = threading.Lock()

_SIGS = {
    "ecg_device_count": (ctypes.c_int, []),
    "ecg_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "ecg_ctx_destroy": (None, [ctypes.c_void_p]),
    "ecg_ctx_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]),
    "ecg_last_error": (ctypes.c_char_p, []),
    "ecg_version": (ctypes.c_char_p, []),
    "ecg_fft": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _u64p, _u64p, ctypes.c_uint32, ABORT_CB, ctypes.c_void_p]),
    "ecg_fft_many": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(_u64p), _u64p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t,
                                    ABORT_CB, ctypes.c_void_p]),
    "ecg_fft_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _u64p, ctypes.c_uint32, ctypes.c_void_p]),
    "ecg_msm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _u64p, _u64p, ctypes.c_size_t, _u64p, ABORT_CB, ctypes.c_void_p]),
    "ecg_msm_multi": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, _u64p, _u64p,
                                     ctypes.c_size_t, _u64p, ABORT_CB, ctypes.c_void_p]),
    "ecg_msm_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "ecg_msm_prepare_bases": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "ecg_msm_prepare_table": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "ecg_point_sum_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, _u64p,
                                         ctypes.c_void_p]),
    "ecg_point_sum": (ctypes.c_int, [ctypes.c_int, _u64p, ctypes.c_size_t, _u64p]),
    "ecg_field_ops": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u64p, _u64p,
                                     ctypes.c_uint32, ctypes.c_size_t, _u64p]),
    "ecg_ec_fft": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _u64p, _u64p, ctypes.c_uint32, ABORT_CB,
                                  ctypes.c_void_p]),
    "ecg_ec_fft_many": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(_u64p), _u64p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t,
                                       ABORT_CB, ctypes.c_void_p]),
    "ecg_ec_fft_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _u64p, ctypes.c_uint32,
                                      ctypes.c_void_p]),
    "ecg_multiple_multiexp": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                             ctypes.c_size_t, ctypes.c_uint32, _u64p]),
    "ecg_msm_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                                  ctypes.c_size_t, _u64p, ctypes.c_int, ctypes.c_size_t, _u64p, ctypes.c_int, _u64p,
                                  ABORT_CB, ctypes.c_void_p]),
    "ecg_base_cache_clear": (None, [ctypes.c_void_p]),
    "ecg_base_cache_keys": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]),
    "ecg_msm_plan_info": (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_int)]),
    "ecg_msm_prepared_stride": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_uint32]),
    "ecg_ctx_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "ecg_msm_chunk_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "ecg_ctx_set_msm_chunk": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "ecg_ctx_set_mem_limit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "ecg_ctx_release_workspace": (ctypes.c_int, [ctypes.c_void_p]),
    "ecg_ec_fft_set_radix": (ctypes.c_int, [ctypes.c_int]),
    "ecg_comm_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_int)]),
    "ecg_comm_last_exchange": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "ecg_runtime_info": (ctypes.c_char_p, []),
    "ecg_msm_table_window": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_size_t]),
    "ecg_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "ecg_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "ecg_comm_destroy": (None, [ctypes.c_void_p]),
    "ecg_comm_allgather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "ecg_comm_alltoall": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "ecg_msm_dist": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    _u64p]),
    "ecg_msm_dist_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_size_t, _u64p, ABORT_CB, ctypes.c_void_p]),
    "ecg_msm_dist_grid": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_size_t, _u64p]),
    "ecg_msm_dist_grid_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_size_t, _u64p, ABORT_CB, ctypes.c_void_p]),
    "ecg_msm_grid_part": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.c_int, ctypes.c_int, _u64p,
                                         ctypes.POINTER(ctypes.c_int)]),
    "ecg_fft_dist": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _u64p, ctypes.c_uint32]),
    "ecg_fft_dist_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _u64p, ctypes.c_uint32,
                                       ABORT_CB, ctypes.c_void_p]),
    "ecg_comm_set_timeout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "ecg_comm_init_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, XCHG_CB, ctypes.c_void_p]),
    "ecg_fft_dist_stage1": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, _u64p,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "ecg_fft_dist_stage3": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_uint32]),
    "ecg_msm_check_bases": (ctypes.c_int, [ctypes.c_int, _u64p, _u64p, ctypes.c_size_t]),
    "ecg_gen_bases_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _u64p, _u64p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_void_p]),
    "ecg_last_kernel_time": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_int)]),
    "ecg_dev_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "ecg_dev_free": (None, [ctypes.c_void_p, ctypes.c_void_p]),
    "ecg_dev_upload": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "ecg_dev_download": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "ecg_device_info": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_char_p, ctypes.c_size_t]),
    "ecg_field_id": (ctypes.c_int, [_u64p, ctypes.c_size_t, ctypes.c_uint32]),
    "ecg_curve_id": (ctypes.c_int, [_u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p, ctypes.c_size_t]),
    "ecg_has_kernel": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "ecg_field_name": (ctypes.c_char_p, [ctypes.c_int]),
    "ecg_curve_name": (ctypes.c_char_p, [ctypes.c_int]),
}

# ag_build::SourceBuilder request kinds (ECG_KIND_*)
KIND_FIELD, KIND_FFT, KIND_EC, KIND_EC_FFT, KIND_MULTIEXP = 0, 1, 2, 3, 4


def lib() -> ctypes.CDLL:
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libecgpu.so not found at {LIB_PATH}: build the HIP extension "
                    f"(`make -C 0g-ec-gpu_amd` or __graft_entry__.build()); there is no CPU fallback")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                if os.environ.get("ECGPU_LIB") and not hasattr(L, name):
                    continue  # an older build under A/B (dev tools): entry points it lacks stay unbound
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def last_error() -> str:
    return lib().ecg_last_error().decode(errors="replace")


def _check(rc: int, what: str = ""):
    if rc == ECG_OK:
        return
    if rc == ECG_ABORTED:
        raise Aborted("GPU call was aborted!")
    raise EcError(f"{what}: {last_error()} (rc={rc})" if what else f"{last_error()} (rc={rc})")


def _ptr(a: np.ndarray):
    if a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError("expected a C-contiguous uint64 array")
    return a.ctypes.data_as(_u64p)


def _abort_cb(maybe_abort: Optional[Callable[[], bool]]):
    if maybe_abort is None:
        return ABORT_CB(0), None  # NULL function pointer
    cb = ABORT_CB(lambda _user: 1 if maybe_abort() else 0)
    return cb, cb  # keep a reference alive for the call


# ---------------------------------------------------------------------------
# SourceBuilder / generate (ag-build/src/source/builder.rs, ag-build/src/lib.rs)
# Kernels are prebuilt for gfx950; the builder records which field/curve
# instantiations a downstream build asked for, and generate() checks that the
# prebuilt library provides them (there is no runtime codegen / nvcc step).
# ---------------------------------------------------------------------------


@dataclass
class SourceBuilder:
    fields: set = field(default_factory=set)
    ffts: set = field(default_factory=set)
    ecs: set = field(default_factory=set)
    ec_ffts: set = field(default_factory=set)
    multiexps: set = field(default_factory=set)
    extra_sources: list = field(default_factory=list)

    @staticmethod
    def new() -> "SourceBuilder":
        return SourceBuilder()

    def add_field(self, f: str) -> "SourceBuilder":
        self.fields.add(f)
        return self

    def add_fft(self, f: str) -> "SourceBuilder":
        self.add_field(f)
        self.ffts.add(f)
        return self

    def add_ec(self, curve: str) -> "SourceBuilder":
        family = curve[:-3] if curve.endswith("_g2") else curve
        if curve.endswith("_g2"):
            self.add_field(family + "_fq2")  # an extension field brings its sub-field (builder.rs:43-55)
        self.add_field(family + "_fq").add_field(family + "_fr")
        self.ecs.add(curve)
        return self

    def add_ec_fft(self, curve: str) -> "SourceBuilder":
        self.add_ec(curve)
        self.ec_ffts.add(curve)
        return self

    def add_multiexp(self, curve: str) -> "SourceBuilder":
        self.add_ec(curve)
        self.multiexps.add(curve)
        return self

    def append_source(self, source: str) -> "SourceBuilder":
        self.extra_sources.append(source)
        return self

    def build_32_bit_limbs(self) -> str:
        return self._describe(32)

    def build_64_bit_limbs(self) -> str:
        return self._describe(64)

    def _describe(self, limb_bits: int) -> str:
        return "\n".join([f"// prebuilt gfx950 kernels, {limb_bits}-bit host limbs"]
                         + [f"// fft {f}" for f in sorted(self.ffts)]
                         + [f"// multiexp {c}" for c in sorted(self.multiexps)])


def generate(sb: SourceBuilder) -> None:
    """ag_build::generate: checks every requested instantiation against the
    loaded library's kernel registry (ecg_has_kernel), as the Rust ag_build
    shim does at build time; an unserved request raises."""
    L = lib()
    requests = ([(KIND_FIELD, f, FIELD_NAMES) for f in sb.fields] + [(KIND_FFT, f, FIELD_NAMES) for f in sb.ffts]
                + [(KIND_EC, c, CURVE_NAMES) for c in sb.ecs] + [(KIND_EC_FFT, c, CURVE_NAMES) for c in sb.ec_ffts]
                + [(KIND_MULTIEXP, c, CURVE_NAMES) for c in sb.multiexps])
    what = {KIND_FIELD: "field", KIND_FFT: "FFT", KIND_EC: "curve", KIND_EC_FFT: "EC-FFT", KIND_MULTIEXP: "multiexp"}
    for kind, name, ids in requests:
        if name not in ids or not L.ecg_has_kernel(kind, ids[name]):
            raise EcError(f"no prebuilt {what[kind]} kernel for {name!r}")


# ---------------------------------------------------------------------------
# Device / Program (rust_gpu_tools::Device, ec_gpu_program::program!)
# ---------------------------------------------------------------------------


class Device:
    def __init__(self, index: int):
        self.index = index

    @staticmethod
    def all() -> list["Device"]:
        return [Device(i) for i in range(lib().ecg_device_count())]

    def _info(self):
        mem, cus, name = ctypes.c_size_t(), ctypes.c_int(), ctypes.create_string_buffer(256)
        _check(lib().ecg_device_info(self.index, ctypes.byref(mem), ctypes.byref(cus), name, 256), "device_info")
        return mem.value, cus.value, name.value.decode()

    def name(self) -> str:
        return f"#{self.index} {self._info()[2]}"

    def memory(self) -> int:
        """Device::memory (bytes of HBM)."""
        return self._info()[0]

    def compute_units(self) -> int:
        return self._info()[1]


class Program:
    """One context per device: device, stream, persistent HBM workspace."""

    def __init__(self, device: Device):
        self.device = device
        h = ctypes.c_void_p()
        _check(lib().ecg_ctx_create(device.index, ctypes.byref(h)), "program!")
        self.handle = h
        self._lock = threading.Lock()

    def device_name(self) -> str:
        return self.device.name()

    def memory(self) -> int:
        mem = ctypes.c_size_t()
        cus = ctypes.c_int()
        _check(lib().ecg_ctx_info(self.handle, ctypes.byref(mem), ctypes.byref(cus)))
        return mem.value

    def compute_units(self) -> int:
        mem = ctypes.c_size_t()
        cus = ctypes.c_int()
        _check(lib().ecg_ctx_info(self.handle, ctypes.byref(mem), ctypes.byref(cus)))
        return cus.value

    def synchronize(self) -> None:
        _check(lib().ecg_ctx_synchronize(self.handle), "synchronize")

    def msm_chunk_size(self, curve="bls12_381") -> int:
        """Terms per MSM device pass (SingleMultiexpKernel::n / calc_chunk_size,
        multiexp.rs:71-93), derived from this device's memory unless pinned."""
        n = ctypes.c_size_t()
        _check(lib().ecg_msm_chunk_size(self.handle, _curve(curve), ctypes.byref(n)), "msm_chunk_size")
        return n.value

    def set_msm_chunk(self, max_terms: int) -> None:
        """Pin the terms per MSM device pass (0 = derived from device memory)."""
        _check(lib().ecg_ctx_set_msm_chunk(self.handle, int(max_terms)), "set_msm_chunk")

    def set_mem_limit(self, nbytes: int) -> None:
        """Cap the memory this context plans with and allocates as scratch
        (ecg_ctx_set_mem_limit; 0 = the device's memory)."""
        _check(lib().ecg_ctx_set_mem_limit(self.handle, int(nbytes)), "set_mem_limit")

    def release_workspace(self):
        """Free this context's device scratch and cached twiddle tables
        (ecg_ctx_release_workspace); later calls regrow what they need."""
        _check(lib().ecg_ctx_release_workspace(self.handle), "release_workspace")

    def kernel_time(self, name: str) -> tuple[float, int]:
        ms = ctypes.c_double()
        cnt = ctypes.c_int()
        _check(lib().ecg_last_kernel_time(self.handle, name.encode(), ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value

    def close(self):
        if getattr(self, "handle", None):
            lib().ecg_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """HBM-resident buffer on a Program's device (DeviceData / upload_multiexp_bases
    analogue).  `ptr` feeds the device-resident entry points."""

    def __init__(self, prog: Program, nbytes: int):
        self.program = prog
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _check(lib().ecg_dev_alloc(prog.handle, self.nbytes, ctypes.byref(p)), "dev_alloc")
        self.ptr = p

    @staticmethod
    def upload(prog: Program, host: np.ndarray) -> "DeviceBuffer":
        h = np.ascontiguousarray(host)
        buf = DeviceBuffer(prog, h.nbytes)
        buf.write(h)
        return buf

    def write(self, host: np.ndarray) -> None:
        h = np.ascontiguousarray(host)
        if h.nbytes > self.nbytes:
            raise EcError("DeviceBuffer.write: host array larger than the buffer")
        _check(lib().ecg_dev_upload(self.program.handle, self.ptr, h.ctypes.data_as(ctypes.c_void_p), h.nbytes))

    def read(self, dtype=np.uint64, shape=None) -> np.ndarray:
        out = np.empty(self.nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        _check(lib().ecg_dev_download(self.program.handle, out.ctypes.data_as(ctypes.c_void_p), self.ptr,
                                      out.nbytes))
        return out.reshape(shape) if shape is not None else out

    def free(self) -> None:
        if self.ptr:
            lib().ecg_dev_free(self.program.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if getattr(self, "program", None) is not None and self.program.handle:
                self.free()
        except Exception:
            pass


def msm_dev(prog: Program, curve, d_bases: DeviceBuffer, d_scalars: DeviceBuffer, n: int) -> np.ndarray:
    """MSM over HBM-resident bases/scalars (ecg_msm_dev) -> Jacobian (3*Lq,)."""
    cid = _curve(curve)
    out = np.zeros(3 * CURVE_FQ_LIMBS[cid], dtype=np.uint64)
    _check(lib().ecg_msm_dev(prog.handle, cid, d_bases.ptr, d_scalars.ptr, n,
                             out.ctypes.data_as(ctypes.c_void_p), 0, None), "msm_dev")
    return out


FOP_ADD, FOP_SUB, FOP_MUL, FOP_SQR, FOP_DOUBLE, FOP_POW, FOP_MONT, FOP_UNMONT, FOP_INV = range(9)


def field_ops(prog: Program, field, form: int, op: int, a: np.ndarray, b: np.ndarray | None = None,
              e: int = 0) -> np.ndarray:
    """ecg_field_ops: one field operation element-wise on the device in one of
    the engine's field forms (0 boundary, 1 product-path reduced radix, 2 an
    Fq's G2 reduced radix) -- the reference's GPU field tests
    (ag-build/src/tests/test_fields.rs).  a, b: (n, limbs) u64 Montgomery."""
    fid = FIELD_NAMES[field] if isinstance(field, str) else int(field)
    a = np.ascontiguousarray(a, dtype=np.uint64)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros_like(a)
    _check(lib().ecg_field_ops(prog.handle, fid, form, op, _ptr(a), _ptr(bb) if bb is not None else None, int(e),
                               a.shape[0], _ptr(out)), "field_ops")
    return out


def msm_grid_part(prog: Program, curve, d_bases: DeviceBuffer, d_scalars: DeviceBuffer, n: int, rank: int,
                  nranks: int) -> tuple[np.ndarray, int]:
    """Rank `rank` of `nranks`'s local step of the grid-split MSM
    (ecg_msm_grid_part): its partial over the full n-term operands and the
    number of Pippenger pieces it ran.  The nranks partials add up to msm_dev."""
    cid = _curve(curve)
    out = np.zeros(3 * CURVE_FQ_LIMBS[cid], dtype=np.uint64)
    pieces = ctypes.c_int(0)
    _check(lib().ecg_msm_grid_part(prog.handle, cid, d_bases.ptr, d_scalars.ptr, n, rank, nranks, _ptr(out),
                                   ctypes.byref(pieces)), "msm_grid_part")
    return out, pieces.value


class PreparedBases(DeviceBuffer):
    """Bases held in the bucket kernels' own layout (ecg_msm_prepare_bases):
    the device-side half of upload_multiexp_bases (ag-cuda-ec/src/multiexp.rs:
    11-19).  Pass it as d_bases / bases_gpu to msm_dev, multiple_multiexp or
    dist.msm_dist; it is immutable and not readable as [x, y] records."""

    def __init__(self, prog: Program, ptr: ctypes.c_void_p, curve_id: int, n: int, window_table: int = 0):
        self.program = prog
        self.ptr = ptr
        self.curve_id = curve_id
        self.n = n
        self.window_table = window_table  # 0, or the window size of the precomputed table
        self.nbytes = 0

    def write(self, host: np.ndarray) -> None:
        raise EcError("PreparedBases are immutable: prepare new bases instead")

    def read(self, dtype=np.uint64, shape=None) -> np.ndarray:
        raise EcError("PreparedBases hold the kernels' internal layout")

    def stride(self) -> int:
        """Bytes per base (all of its window-table rows)."""
        wt = self.window_table if self.window_table > 0 else 0
        if self.window_table < 0:
            raise EcError("PreparedBases.stride: automatic window table (pass the window size to prepare_bases)")
        return int(lib().ecg_msm_prepared_stride(self.curve_id, wt))

    def view(self, start: int, count: int | None = None) -> "PreparedView":
        """Bases start.. of this buffer in the same form (a base-aligned
        pointer into it, e.g. one rank's shard); no copy.  The view borrows
        this buffer: keep it alive while the view is used."""
        count = self.n - start if count is None else count
        if not (0 <= start and 0 <= count and start + count <= self.n):
            raise EcError(f"PreparedBases.view: [{start}, {start + count}) outside [0, {self.n})")
        return PreparedView(self, start, count)

    def free(self) -> None:
        if self.ptr:
            lib().ecg_dev_free(self.program.handle, self.ptr)
            self.ptr = None


class PreparedView(PreparedBases):
    """Base-aligned slice of PreparedBases (does not own memory)."""

    def __init__(self, parent: PreparedBases, start: int, count: int):
        self._parent = parent
        super().__init__(parent.program, ctypes.c_void_p(parent.ptr.value + start * parent.stride()),
                         parent.curve_id, count, parent.window_table)

    def free(self) -> None:  # the parent owns the allocation
        self.ptr = None

    def __del__(self):
        pass


def prepare_bases(prog: Program, curve, d_bases: DeviceBuffer, n: int, window_table=None) -> PreparedBases:
    """Convert n HBM-resident [x, y] bases once into the kernels' layout
    (ecg_msm_prepare_bases); the MSMs over the result skip that conversion.
    window_table: None = plain records; 0 = precompute the window table for
    n-term MSMs (window chosen by the engine); c = table of window size c
    (ecg_msm_prepare_table, G1 only)."""
    cid = _curve(curve)
    p = ctypes.c_void_p()
    if window_table is None:
        _check(lib().ecg_msm_prepare_bases(prog.handle, cid, d_bases.ptr, n, ctypes.byref(p)), "prepare_bases")
        return PreparedBases(prog, p, cid, n)
    _check(lib().ecg_msm_prepare_table(prog.handle, cid, d_bases.ptr, n, int(window_table), ctypes.byref(p)),
           "prepare_table")
    return PreparedBases(prog, p, cid, n, window_table=int(window_table) or -1)


def fft_dev(prog: Program, field, d_data: DeviceBuffer, omega: np.ndarray, log_n: int) -> None:
    """In-place NTT of HBM-resident data (ecg_fft_dev)."""
    fid = _fft_field(field)
    om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
    _check(lib().ecg_fft_dev(prog.handle, fid, d_data.ptr, _ptr(om), log_n, None), "fft_dev")


def gen_bases_dev(prog: Program, curve, a: int, b: int, n: int) -> DeviceBuffer:
    """Synthetic bases P_i = (a + i b) G generated on the device."""
    cid = _curve(curve)
    buf = DeviceBuffer(prog, n * 2 * CURVE_FQ_LIMBS[cid] * 8)
    au = np.array([(a >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
    bu = np.array([(b >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
    _check(lib().ecg_gen_bases_dev(prog.handle, cid, _ptr(au), _ptr(bu), n, buf.ptr, None), "gen_bases")
    return buf


# ---------------------------------------------------------------------------
# ag-cuda-ec batched multi-line MSM (ag-cuda-ec/src/multiexp.rs)
# ---------------------------------------------------------------------------


def upload_multiexp_bases(prog: Program, bases: np.ndarray, curve=None, window_table=None):
    """ag_cuda_ec::multiexp::upload_multiexp_bases (multiexp.rs:11-19): affine
    bases (n, 2*Lq) u64, Montgomery x||y, identity = zeros (GpuRepr) -> HBM.
    With `curve` given, the upload is also converted once into the kernels'
    layout (prepare_bases, optionally with a window table) and the
    PreparedBases are returned."""
    raw = DeviceBuffer.upload(prog, np.ascontiguousarray(bases, dtype=np.uint64))
    if curve is None:
        return raw
    prep = prepare_bases(prog, curve, raw, np.asarray(bases).shape[0], window_table=window_table)
    raw.free()
    return prep


def multiple_multiexp(prog: Program, bases_gpu: DeviceBuffer, exponents, num_chunks: int,
                      window_size: int = 0, neg_is_cheap: bool = True, curve="bls12_381",
                      pin_window: bool = False, exps_montgomery: bool = False) -> np.ndarray:
    """ag_cuda_ec::multiexp::multiple_multiexp (multiexp.rs:21-81).

    bases_gpu holds n_lines * len(exponents) bases; `exponents` is one row of
    canonical scalars ((line_len, 4) u64 host array, or a DeviceBuffer plus
    line_len via a (buffer, line_len) tuple).  Returns (n_lines * num_chunks,
    3*Lq) normalised Jacobian points, result[line * num_chunks + chunk].
    window_size / neg_is_cheap are the reference kernel's tuning knobs; results
    never depend on them.  The engine picks its own window unless
    pin_window=True (then window_size in 1..22 is used as is).
    exps_montgomery=True takes Fr elements in Montgomery form and runs the
    to_bigint conversion (benches/amt.rs:25-26, on the CPU there) on device."""
    cid = _curve(curve)
    lq = CURVE_FQ_LIMBS[cid]
    if isinstance(exponents, tuple):
        dbuf, line_len = exponents
        sc_ptr, on_dev = dbuf.ptr, 1
        keep = None
    else:
        keep = np.ascontiguousarray(exponents, dtype=np.uint64).reshape(-1, 4)
        line_len = keep.shape[0]
        sc_ptr, on_dev = keep.ctypes.data_as(ctypes.c_void_p), 0
    if line_len == 0:
        raise EcError("multiple_multiexp: empty exponent row")
    n_bases = bases_gpu.n if isinstance(bases_gpu, PreparedBases) else bases_gpu.nbytes // (2 * lq * 8)
    n_lines = n_bases // line_len
    out = np.zeros((n_lines * num_chunks, 3 * lq), dtype=np.uint64)
    wb = int(window_size) if pin_window else 0
    _check(lib().ecg_multiple_multiexp(prog.handle, cid, bases_gpu.ptr, n_lines * line_len, sc_ptr, on_dev,
                                       int(exps_montgomery), line_len, num_chunks, wb, _ptr(out)),
           "multiple_multiexp")
    del keep
    return out


def program(device: Device) -> Program:
    """ec_gpu_program::program!(device)."""
    return Program(device)


load_program = program  # ec_gpu_program::load_program! (test-tools)


# ---------------------------------------------------------------------------
# FFT (ec-gpu-proxy/src/fft.rs)
# ---------------------------------------------------------------------------


def _fft_field(f) -> int:
    fid = FIELD_NAMES.get(f, f) if isinstance(f, str) else int(f)
    if fid not in (FIELD_BLS12_381_FR, FIELD_BN254_FR):
        raise EcError(f"FftKernel: unsupported field {f!r}")
    return fid


class SingleFftKernel:
    def __init__(self, prog: Program, fid: int, maybe_abort=None):
        self.program = prog
        self.fid = fid
        self.maybe_abort = maybe_abort

    def radix_fft(self, inp: np.ndarray, omega: np.ndarray, log_n: int) -> None:
        """In place: inp (2^log_n, 4) uint64 Montgomery."""
        if inp.shape != (1 << log_n, 4):
            raise EcError(f"radix_fft: expected shape {(1 << log_n, 4)}, got {inp.shape}")
        om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
        cb, keep = _abort_cb(self.maybe_abort)
        with self.program._lock:
            rc = lib().ecg_fft(self.program.handle, self.fid, _ptr(inp), _ptr(om), log_n, cb, None)
        del keep
        _check(rc, "radix_fft")


class FftKernel:
    """One FFT kernel per device (fft.rs:139-246)."""

    def __init__(self, kernels: list[SingleFftKernel]):
        self.kernels = kernels

    @staticmethod
    def create(programs: Sequence[Program], field: str | int = "bls12_381_fr") -> "FftKernel":
        return FftKernel._create(programs, field, None)

    @staticmethod
    def create_with_abort(programs, maybe_abort: Callable[[], bool], field: str | int = "bls12_381_fr"):
        return FftKernel._create(programs, field, maybe_abort)

    @staticmethod
    def _create(programs, field, maybe_abort):
        fid = _fft_field(field)
        kernels = [SingleFftKernel(p, fid, maybe_abort) for p in programs]
        if not kernels:
            raise EcError("No working GPUs found!")
        return FftKernel(kernels)

    def radix_fft(self, inp: np.ndarray, omega: np.ndarray, log_n: int) -> None:
        """Uses the first GPU (fft.rs:200-204)."""
        self.kernels[0].radix_fft(inp, omega, log_n)

    def radix_fft_many(self, inputs: Sequence[np.ndarray], omegas: Sequence[np.ndarray],
                       log_ns: Sequence[int]) -> None:
        """ceil(m / #devices) chunks, one host thread per device, first error
        wins and stops the other workers at their next input (fft.rs:211-246)."""
        n = len(inputs)
        if not (len(omegas) == n and len(log_ns) == n):
            raise EcError("radix_fft_many: inputs/omegas/log_ns length mismatch")
        if n == 0:
            return
        for a, ln in zip(inputs, log_ns):
            if a.shape != (1 << ln, 4) or a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
                raise EcError("radix_fft_many: each input must be a C-contiguous (2^log_n, 4) uint64 array")
        nd = len(self.kernels)
        ctxs = (ctypes.c_void_p * nd)(*[k.program.handle.value for k in self.kernels])
        ptrs = (_u64p * n)(*[_ptr(a) for a in inputs])
        om = np.ascontiguousarray(np.stack([np.asarray(o, dtype=np.uint64).reshape(4) for o in omegas]))
        lns = (ctypes.c_uint32 * n)(*log_ns)
        cb, keep = _abort_cb(self.kernels[0].maybe_abort)
        rc = lib().ecg_fft_many(ctxs, nd, self.kernels[0].fid, ptrs, _ptr(om), lns, n, cb, None)
        del keep
        _check(rc, "radix_fft_many")


# ---------------------------------------------------------------------------
# EC-FFT over G1 (ec-gpu-proxy/src/ec_fft.rs, ag-cuda-ec/src/ec_fft.rs)
# ---------------------------------------------------------------------------


def _jac_shape(cid: int, log_n: int):
    return (1 << log_n, 3 * CURVE_FQ_LIMBS[cid])


class SingleEcFftKernel:
    def __init__(self, prog: Program, cid: int, maybe_abort=None):
        self.program = prog
        self.cid = cid
        self.maybe_abort = maybe_abort

    def radix_ec_fft(self, inp: np.ndarray, omega: np.ndarray, log_n: int) -> None:
        """In place (ec_fft.rs:56-164): inp (2^log_n, 3*Lq) uint64 Jacobian points
        (G::Curve, Montgomery), rewritten normalised; omega Fr Montgomery."""
        if inp.shape != _jac_shape(self.cid, log_n) or inp.dtype != np.uint64 or not inp.flags["C_CONTIGUOUS"]:
            raise EcError(f"radix_ec_fft: expected a C-contiguous uint64 array of shape {_jac_shape(self.cid, log_n)}")
        om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
        cb, keep = _abort_cb(self.maybe_abort)
        with self.program._lock:
            rc = lib().ecg_ec_fft(self.program.handle, self.cid, _ptr(inp), _ptr(om), log_n, cb, None)
        del keep
        _check(rc, "radix_ec_fft")


class EcFftKernel:
    """One EC-FFT kernel per device (ec_fft.rs:167-271)."""

    def __init__(self, kernels: list[SingleEcFftKernel]):
        self.kernels = kernels

    @staticmethod
    def create(programs: Sequence[Program], curve: str | int = "bls12_381") -> "EcFftKernel":
        return EcFftKernel._create(programs, curve, None)

    @staticmethod
    def create_with_abort(programs, maybe_abort: Callable[[], bool], curve: str | int = "bls12_381"):
        return EcFftKernel._create(programs, curve, maybe_abort)

    @staticmethod
    def _create(programs, curve, maybe_abort):
        cid = _curve(curve)
        kernels = [SingleEcFftKernel(p, cid, maybe_abort) for p in programs]
        if not kernels:
            raise EcError("No working GPUs found!")
        return EcFftKernel(kernels)

    def radix_ec_fft(self, inp: np.ndarray, omega: np.ndarray, log_n: int) -> None:
        """Uses the first GPU (ec_fft.rs:213-217)."""
        self.kernels[0].radix_ec_fft(inp, omega, log_n)

    def radix_ec_fft_many(self, inputs: Sequence[np.ndarray], omegas: Sequence[np.ndarray],
                          log_ns: Sequence[int]) -> None:
        """ceil(m / #devices) transforms per device, first error wins (ec_fft.rs:224-270)."""
        n = len(inputs)
        if not (len(omegas) == n and len(log_ns) == n):
            raise EcError("radix_ec_fft_many: inputs/omegas/log_ns length mismatch")
        if n == 0:
            return
        cid = self.kernels[0].cid
        for a, ln in zip(inputs, log_ns):
            if a.shape != _jac_shape(cid, ln) or a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
                raise EcError("radix_ec_fft_many: each input must be a C-contiguous (2^log_n, 3*Lq) uint64 array")
        nd = len(self.kernels)
        ctxs = (ctypes.c_void_p * nd)(*[k.program.handle.value for k in self.kernels])
        ptrs = (_u64p * n)(*[_ptr(a) for a in inputs])
        om = np.ascontiguousarray(np.stack([np.asarray(o, dtype=np.uint64).reshape(4) for o in omegas]))
        lns = (ctypes.c_uint32 * n)(*log_ns)
        cb, keep = _abort_cb(self.kernels[0].maybe_abort)
        rc = lib().ecg_ec_fft_many(ctxs, nd, cid, ptrs, _ptr(om), lns, n, cb, None)
        del keep
        _check(rc, "radix_ec_fft_many")


def radix_ec_fft(prog: Program, inp: np.ndarray, omegas, curve="bls12_381") -> None:
    """ag_cuda_ec::ec_fft::radix_ec_fft (ag-cuda-ec/src/ec_fft.rs:12-93): in
    place, n = len(inp) a power of two; omegas[0] is the n-th root of unity
    (the reference passes [omega, omega^2, omega^4, ...])."""
    n = inp.shape[0]
    log_n = n.bit_length() - 1
    if n != 1 << log_n:
        raise EcError("radix_ec_fft: input length must be a power of two")
    SingleEcFftKernel(prog, _curve(curve)).radix_ec_fft(inp, np.asarray(omegas, dtype=np.uint64).reshape(-1, 4)[0],
                                                        log_n)


def ec_fft_set_radix(max_log_radix: int) -> None:
    """Largest log2-radix of the EC-FFT stages, process-wide (ecg_ec_fft_set_radix):
    1 = radix-2 stages only, 0 = the engine's choice per size.  Results never
    depend on it."""
    _check(lib().ecg_ec_fft_set_radix(int(max_log_radix)), "ec_fft_set_radix")


def ec_fft_dev(prog: Program, curve, d_data: DeviceBuffer, omega: np.ndarray, log_n: int) -> None:
    """In-place EC-FFT of HBM-resident Jacobian points (ecg_ec_fft_dev)."""
    om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
    _check(lib().ecg_ec_fft_dev(prog.handle, _curve(curve), d_data.ptr, _ptr(om), log_n, None), "ec_fft_dev")


# ---------------------------------------------------------------------------
# Multiexp (ec-gpu-proxy/src/multiexp.rs)
# ---------------------------------------------------------------------------


class Worker:
    """threadpool::Worker stand-in (the device work is dispatched by the C++
    library with one host thread per device)."""

    def __init__(self, num_threads: Optional[int] = None):
        env = os.environ.get("EC_GPU_NUM_THREADS")
        self.num_threads = num_threads or (int(env) if env and env.isdigit() else (os.cpu_count() or 1))

    def log_num_threads(self) -> int:
        return max(0, self.num_threads.bit_length() - 1)


def _curve(c) -> int:
    cid = CURVE_NAMES.get(c, c) if isinstance(c, str) else int(c)
    if cid not in CURVE_FQ_LIMBS:
        raise EcError(f"MultiexpKernel: unsupported curve {c!r}")
    return cid


class FullDensity:
    """QueryDensity with every base present (multiexp_cpu.rs:96-115)."""

    def generate_exps(self, exponents: np.ndarray) -> np.ndarray:
        return exponents

    def get_query_size(self):
        return None


class DensityTracker:
    """bellman/ec-gpu DensityTracker (multiexp_cpu.rs:117-207): a bit per
    exponent; set bits consume the (compacted) bases in order.  The product
    path hands the packed bitmap to the device (`words()`); generate_exps here
    is the host restatement used for inspection only."""

    def __init__(self, bits=None):
        self.bv = [] if bits is None else [bool(b) for b in bits]
        self.total_density = sum(self.bv)

    @staticmethod
    def new() -> "DensityTracker":
        return DensityTracker()

    def add_element(self) -> None:
        self.bv.append(False)

    def inc(self, idx: int) -> None:
        if not self.bv[idx]:
            self.bv[idx] = True
            self.total_density += 1

    def get_total_density(self) -> int:
        return self.total_density

    def get_query_size(self) -> int:
        return len(self.bv)

    def extend(self, other: "DensityTracker", is_input_density: bool) -> None:
        """multiexp_cpu.rs:162-206, including the coalesced first input."""
        if not other.bv:
            return
        if not self.bv:
            self.total_density = other.total_density
            self.bv = list(other.bv)
            return
        if is_input_density:
            if other.bv[0]:
                if self.bv[0]:
                    self.total_density -= 1
                else:
                    self.bv[0] = True
            self.bv.extend(other.bv[1:])
        else:
            self.bv.extend(other.bv)
        self.total_density += other.total_density

    def words(self, n: int | None = None) -> np.ndarray:
        """bitvec<usize, Lsb0> storage: bit i -> word i/64, bit i%64."""
        n = len(self.bv) if n is None else n
        bits = np.zeros(((n + 63) // 64) * 64, dtype=np.uint8)
        m = min(n, len(self.bv))
        bits[:m] = np.asarray(self.bv[:m], dtype=np.uint8)
        return np.ascontiguousarray(np.packbits(bits, bitorder="little").view(np.uint64))

    def clone(self) -> "DensityTracker":
        d = DensityTracker(self.bv)
        d.total_density = self.total_density
        return d

    def __eq__(self, other) -> bool:  # #[derive(PartialEq)]: bv and total_density
        return isinstance(other, DensityTracker) and self.bv == other.bv and \
            self.total_density == other.total_density

    def generate_exps(self, exponents: np.ndarray) -> np.ndarray:
        keep = np.asarray(self.bv[:len(exponents)], dtype=bool)
        return exponents[:len(keep)][keep]


class SingleMultiexpKernel:
    def __init__(self, prog: Program, cid: int, maybe_abort=None):
        self.program = prog
        self.cid = cid
        self.maybe_abort = maybe_abort

    @property
    def n(self) -> int:
        """Terms per device pass (multiexp.rs:61-63 `n`, from calc_chunk_size);
        longer inputs run as several passes inside one call."""
        return self.program.msm_chunk_size(self.cid)

    def multiexp(self, bases: np.ndarray, exps: np.ndarray) -> np.ndarray:
        lq = CURVE_FQ_LIMBS[self.cid]
        if bases.shape[0] != exps.shape[0]:
            raise EcError("multiexp: bases and exponents differ in length")
        b = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, 2 * lq)
        e = np.ascontiguousarray(exps, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros(3 * lq, dtype=np.uint64)
        cb, keep = _abort_cb(self.maybe_abort)
        with self.program._lock:
            rc = lib().ecg_msm(self.program.handle, self.cid, _ptr(b), _ptr(e), e.shape[0], _ptr(out), cb, None)
        del keep
        _check(rc, "multiexp")
        return out


class MultiexpKernel:
    """Multiexp kernels for several devices (multiexp.rs:256-404)."""

    def __init__(self, kernels: list[SingleMultiexpKernel]):
        self.kernels = kernels

    @staticmethod
    def create(programs: Sequence[Program], devices: Sequence[Device] = (), curve: str | int = "bls12_381"):
        return MultiexpKernel._create(programs, curve, None)

    @staticmethod
    def create_with_abort(programs, devices, maybe_abort: Callable[[], bool], curve: str | int = "bls12_381"):
        return MultiexpKernel._create(programs, curve, maybe_abort)

    @staticmethod
    def _create(programs, curve, maybe_abort):
        cid = _curve(curve)
        kernels = [SingleMultiexpKernel(p, cid, maybe_abort) for p in programs]
        if not kernels:
            raise EcError("No working GPUs found!")
        return MultiexpKernel(kernels)

    def num_kernels(self) -> int:
        return len(self.kernels)

    def multiexp(self, pool: Worker, bases: np.ndarray, exps: np.ndarray, skip: int = 0) -> np.ndarray:
        """sum_i exps[i] * bases[skip + i]  ->  Jacobian (3*Lq,) uint64."""
        cid = self.kernels[0].cid
        lq = CURVE_FQ_LIMBS[cid]
        e = np.ascontiguousarray(exps, dtype=np.uint64).reshape(-1, 4)
        n = e.shape[0]
        if skip + n > bases.shape[0]:
            raise EcError("multiexp: Expected more bases from source.")
        b = np.ascontiguousarray(bases[skip:skip + n], dtype=np.uint64).reshape(-1, 2 * lq)
        out = np.zeros(3 * lq, dtype=np.uint64)
        nd = len(self.kernels)
        ctxs = (ctypes.c_void_p * nd)(*[k.program.handle.value for k in self.kernels])
        cb, keep = _abort_cb(self.kernels[0].maybe_abort)
        rc = lib().ecg_msm_multi(ctxs, nd, cid, _ptr(b), _ptr(e), n, _ptr(out), cb, None)
        del keep
        _check(rc, "multiexp")
        return out

    def multiexp_ex(self, bases: np.ndarray, exps: np.ndarray, skip: int = 0, density=None,
                    exps_montgomery: bool = False, ark_affine: bool = False, cache_bases: bool = False) -> np.ndarray:
        """multiexp with the reference's host prep moved on device (ecg_msm_ex,
        first device): density-filtered exps (DensityTracker), Montgomery Fr
        exps, arkworks Affine{x,y,infinity} bases ((n, 2*Lq+1) uint64 records),
        and an optional persistent base cache."""
        k = self.kernels[0]
        cid = k.cid
        lq = CURVE_FQ_LIMBS[cid]
        rec = 2 * lq + 1 if ark_affine else 2 * lq
        b = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, rec)
        if cache_bases:
            # the cache is keyed by the host address: cache only the caller's
            # own array (never a temporary copy), and keep it alive while cached
            if not isinstance(bases, np.ndarray) or not np.shares_memory(b, bases):
                raise EcError("multiexp_ex(cache_bases=True) needs a C-contiguous uint64 bases array "
                              "(a converted copy cannot be cached by address)")
            pins = k.program.__dict__.setdefault("_base_pins", {})
            pins[b.ctypes.data] = bases  # keeps the cached array alive (the cache holds its address)
        e = np.ascontiguousarray(exps, dtype=np.uint64).reshape(-1, 4)
        dens = None
        if density is not None and not isinstance(density, FullDensity):
            dens = density.words(e.shape[0])
        out = np.zeros(3 * lq, dtype=np.uint64)
        cb, keep = _abort_cb(k.maybe_abort)
        with k.program._lock:
            rc = lib().ecg_msm_ex(k.program.handle, cid, b.ctypes.data_as(ctypes.c_void_p), int(ark_affine),
                                  b.shape[0], skip, _ptr(e), int(exps_montgomery), e.shape[0],
                                  _ptr(dens) if dens is not None else None, int(cache_bases), _ptr(out), cb, None)
        del keep
        if "_base_pins" in k.program.__dict__:
            _prune_base_pins(k.program)
        _check(rc, "multiexp")
        return out

    def clear_base_cache(self) -> None:
        for k in self.kernels:
            lib().ecg_base_cache_clear(k.program.handle)
            k.program.__dict__.pop("_base_pins", None)


def _prune_base_pins(prog: Program) -> None:
    """Drop the references to host arrays the C base cache no longer holds
    (evicted as the oldest of its 8 entries, or replaced after a content
    change at the same address), so they are not kept alive for the life of
    the Program."""
    cap = 64
    keys = (ctypes.c_void_p * cap)()
    n = lib().ecg_base_cache_keys(prog.handle, keys, cap)
    live = {keys[i] for i in range(min(n, cap))}
    pins = prog.__dict__.get("_base_pins", {})
    for addr in [a for a in pins if a not in live]:
        del pins[addr]


def msm_plan(curve, n: int, window_bits: int = 0) -> tuple[int, int, str]:
    """(c, windows, sort) of a one-task MSM of n terms (ecg_msm_plan_info):
    sort is "global", "pw_one" (one sort over every window block) or
    "pw_block" (one sort per window block)."""
    c, w, mode = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
    _check(lib().ecg_msm_plan_info(_curve(curve), int(n), int(window_bits), ctypes.byref(c), ctypes.byref(w),
                                   ctypes.byref(mode)), "msm_plan")
    return c.value, w.value, {0: "global", 1: "pw_one", 2: "pw_block"}[mode.value]


def check_bases(curve, bases: np.ndarray, exps: np.ndarray) -> None:
    """Raise EcError like multiexp_cpu.rs:57-61 if a base with a non-zero
    exponent is the identity."""
    cid = _curve(curve)
    b = np.ascontiguousarray(bases, dtype=np.uint64)
    e = np.ascontiguousarray(exps, dtype=np.uint64)
    _check(lib().ecg_msm_check_bases(cid, _ptr(b), _ptr(e), e.size // 4), "multiexp")
