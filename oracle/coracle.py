"""ctypes binding of the C oracle (oracle/oracle.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / timed CPU baseline.  Never imported by the product package.
Arrays are numpy uint64 in the reference's in-memory layout: little-endian u64
limbs, Montgomery form for field elements (ark_ff::Fp), canonical for scalars
(BigInt<4>), bases as [x, y] (GpuRepr, identity = zeros).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

FIELD_IDS = {"bls12_381_fr": 0, "bls12_381_fq": 1, "bn254_fr": 2, "bn254_fq": 3}
CURVE_IDS = {"bls12_381": 0, "bn254": 1}
CURVE_FQ = {0: 1, 1: 3}
CURVE_FR = {0: 0, 1: 2}

_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i, u32, sz, u64 = ctypes.c_int, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_uint64
        sig = {
            "orc_field_limbs": (i, [i]),
            "orc_fmul": (None, [i, _u64p, _u64p, _u64p]),
            "orc_fadd": (None, [i, _u64p, _u64p, _u64p]),
            "orc_fsub": (None, [i, _u64p, _u64p, _u64p]),
            "orc_finv": (None, [i, _u64p, _u64p]),
            "orc_to_mont": (None, [i, _u64p, _u64p]),
            "orc_from_mont": (None, [i, _u64p, _u64p]),
            "orc_pow_u64": (None, [i, _u64p, _u64p, u64]),
            "orc_serial_fft": (None, [i, _u64p, _u64p, u32]),
            "orc_parallel_fft": (i, [i, _u64p, _u64p, u32, u32]),
            "orc_poly_eval": (None, [i, _u64p, sz, _u64p, _u64p]),
            "orc_multiexp_cpu": (i, [i, _u64p, _u64p, sz, _u64p, i, u32]),
            "orc_naive_multiexp": (None, [i, _u64p, _u64p, sz, _u64p]),
            "orc_jac_double": (None, [i, _u64p, _u64p]),
            "orc_jac_add": (None, [i, _u64p, _u64p, _u64p]),
            "orc_jac_add_mixed": (None, [i, _u64p, _u64p, _u64p]),
            "orc_jac_to_affine": (i, [i, _u64p, _u64p]),
            "orc_gen_mul": (None, [i, _u64p, _u64p]),
            "orc_gen_bases": (None, [i, _u64p, _u64p, sz, _u64p, i]),
            "orc_kat_scalar": (None, [i, _u64p, _u64p, _u64p, sz, _u64p, i]),
            "orc_serial_ec_fft": (None, [i, _u64p, _u64p, u32, i]),
            "orc_naive_ec_dft": (None, [i, _u64p, _u64p, u32, _u64p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u64p)


def u64arr(values, n) -> np.ndarray:
    """ints -> (len, n) uint64 little-endian limbs."""
    out = np.zeros((len(values), n), dtype=np.uint64)
    for k, v in enumerate(values):
        for i in range(n):
            out[k, i] = (v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return out


def to_ints(a: np.ndarray) -> list[int]:
    a = np.asarray(a, dtype=np.uint64).reshape(-1, a.shape[-1])
    return [sum(int(v) << (64 * i) for i, v in enumerate(row)) for row in a]


def limbs(fid: int) -> int:
    return lib().orc_field_limbs(fid)


def to_mont(fid: int, a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, limbs(fid))
    out = np.empty_like(a)
    for k in range(a.shape[0]):
        lib().orc_to_mont(fid, ptr(out[k]), ptr(a[k]))
    return out


def from_mont(fid: int, a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, limbs(fid))
    out = np.empty_like(a)
    for k in range(a.shape[0]):
        lib().orc_from_mont(fid, ptr(out[k]), ptr(a[k]))
    return out


def serial_fft(fid: int, a: np.ndarray, omega: np.ndarray, log_n: int) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64).copy()
    lib().orc_serial_fft(fid, ptr(a), ptr(np.ascontiguousarray(omega, dtype=np.uint64)), log_n)
    return a


def parallel_fft(fid: int, a: np.ndarray, omega: np.ndarray, log_n: int, log_threads: int) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64).copy()
    rc = lib().orc_parallel_fft(fid, ptr(a), ptr(np.ascontiguousarray(omega, dtype=np.uint64)),
                                log_n, log_threads)
    if rc != 0:
        raise ValueError("parallel_fft failed: %d" % rc)
    return a


def poly_eval(fid: int, a: np.ndarray, x: np.ndarray) -> np.ndarray:
    """sum_j a_j x^j (Montgomery in and out): one DFT output X_k = P(omega^k)."""
    a = np.ascontiguousarray(a, dtype=np.uint64)
    out = np.zeros(limbs(fid), dtype=np.uint64)
    lib().orc_poly_eval(fid, ptr(a), a.shape[0], ptr(np.ascontiguousarray(x, dtype=np.uint64)), ptr(out))
    return out


class IdentityBaseError(ValueError):
    pass


def multiexp_cpu(cid: int, bases: np.ndarray, exps: np.ndarray, nthreads: int = 1, c: int = 0) -> np.ndarray:
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    exps = np.ascontiguousarray(exps, dtype=np.uint64)
    nq = limbs(CURVE_FQ[cid])
    out = np.zeros(3 * nq, dtype=np.uint64)
    rc = lib().orc_multiexp_cpu(cid, ptr(bases), ptr(exps), exps.size // 4, ptr(out), nthreads, c)
    if rc == -3:
        raise IdentityBaseError("Encountered an identity element in the CRS.")
    if rc != 0:
        raise RuntimeError("orc_multiexp_cpu failed: %d" % rc)
    return out


def naive_multiexp(cid: int, bases: np.ndarray, exps: np.ndarray) -> np.ndarray:
    nq = limbs(CURVE_FQ[cid])
    out = np.zeros(3 * nq, dtype=np.uint64)
    lib().orc_naive_multiexp(cid, ptr(np.ascontiguousarray(bases, dtype=np.uint64)),
                             ptr(np.ascontiguousarray(exps, dtype=np.uint64)), exps.size // 4, ptr(out))
    return out


def jac_to_affine(cid: int, jac: np.ndarray):
    """Returns (x, y) Montgomery uint64 arrays, or None for the identity."""
    nq = limbs(CURVE_FQ[cid])
    xy = np.zeros(2 * nq, dtype=np.uint64)
    inf = lib().orc_jac_to_affine(cid, ptr(xy), ptr(np.ascontiguousarray(jac, dtype=np.uint64)))
    return None if inf else xy


def gen_mul(cid: int, k: int) -> np.ndarray:
    nq = limbs(CURVE_FQ[cid])
    out = np.zeros(3 * nq, dtype=np.uint64)
    lib().orc_gen_mul(cid, ptr(u64arr([k], 4)[0]), ptr(out))
    return out


def gen_bases(cid: int, a: int, b: int, n: int, nthreads: int = 8) -> np.ndarray:
    nq = limbs(CURVE_FQ[cid])
    out = np.zeros((n, 2 * nq), dtype=np.uint64)
    lib().orc_gen_bases(cid, ptr(u64arr([a], 4)[0]), ptr(u64arr([b], 4)[0]), n, ptr(out), nthreads)
    return out


def kat_scalar(cid: int, a: int, b: int, scalars: np.ndarray, nthreads: int = 8) -> int:
    out = np.zeros(4, dtype=np.uint64)
    sc = np.ascontiguousarray(scalars, dtype=np.uint64)
    lib().orc_kat_scalar(cid, ptr(u64arr([a], 4)[0]), ptr(u64arr([b], 4)[0]), ptr(sc), sc.size // 4,
                         ptr(out), nthreads)
    return to_ints(out.reshape(1, 4))[0]


def serial_ec_fft(cid: int, pts: np.ndarray, omega: np.ndarray, log_n: int, nthreads: int = 8) -> np.ndarray:
    """serial_ec_fft (ec_fft_cpu.rs:12-56) on (n, 3*Lq) Jacobian points; returns a copy."""
    a = np.array(pts, dtype=np.uint64, order="C", copy=True)
    lib().orc_serial_ec_fft(cid, ptr(a), ptr(np.ascontiguousarray(omega, dtype=np.uint64)), log_n, nthreads)
    return a


def naive_ec_dft(cid: int, pts: np.ndarray, omega: np.ndarray, log_n: int) -> np.ndarray:
    a = np.ascontiguousarray(pts, dtype=np.uint64)
    out = np.zeros_like(a)
    lib().orc_naive_ec_dft(cid, ptr(a), ptr(np.ascontiguousarray(omega, dtype=np.uint64)), log_n, ptr(out))
    return out
