"""Pure-Python big-int restatement of the reference CPU algorithms.

TEST INFRASTRUCTURE ONLY.  Nothing on the product path imports this module;
only ``tests/``, ``tests/golden/make_golden.py``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may use it, and only as the checker.

It is deliberately written from the *mathematical* definitions with Python
integers (no limbs, no Montgomery tricks except the R = 2^(64*N) layout
convention) so that it is an independent implementation from the C oracle
(``oracle/oracle.c``) and from the HIP kernels.

Restated reference functions (paths relative to the reference repo):

* ``serial_fft``      -- ec-gpu-proxy/src/fft_cpu.rs:10-52
* ``parallel_fft``    -- ec-gpu-proxy/src/fft_cpu.rs:59-111
* ``pow_vartime``     -- ec-gpu-proxy/src/lib.rs:26-39
* ``multiexp_cpu``    -- ec-gpu-proxy/src/multiexp_cpu.rs:244-367
  (window c = 3 if N < 32 else ceil(ln N), windows over MODULUS_BIT_SIZE,
  exp==0 skipped, exp==1 added directly in window 0, identity bases rejected,
  summation by parts, MSB-first fold with c doublings)
* Jacobian formulas   -- ag-build/cl/ec.cl:17-120 (dbl-2009-l, madd-2007-bl,
  add-2007-bl) -- used by ``jac_*`` below
* ``omega(n)``        -- ec-gpu-proxy/tests/fft.rs:16-24
* ``GpuField``/``GpuRepr`` layouts -- ag-types/src/impls.rs:26-58
"""
from __future__ import annotations

import math
from dataclasses import dataclass

# --------------------------------------------------------------------------
# Parameter sets (ark-bls12-381 0.4 / ark-bn254 0.4 public curve constants)
# --------------------------------------------------------------------------


@dataclass(frozen=True)
class Field:
    name: str
    modulus: int
    limbs64: int           # N in ark_ff::Fp<MontBackend<_, N>, N>
    generator: int = 0     # multiplicative generator (FftField::GENERATOR)
    two_adicity: int = 0

    @property
    def R(self) -> int:  # Montgomery radix, R = 2^(64 N) exactly as arkworks
        return 1 << (64 * self.limbs64)

    @property
    def bits(self) -> int:  # PrimeField::MODULUS_BIT_SIZE
        return self.modulus.bit_length()

    def to_mont(self, x: int) -> int:
        return (x % self.modulus) * self.R % self.modulus

    def from_mont(self, x: int) -> int:
        return x * pow(self.R, -1, self.modulus) % self.modulus

    def two_adic_root(self) -> int:
        t = (self.modulus - 1) >> self.two_adicity
        return pow(self.generator, t, self.modulus)

    def omega(self, n: int) -> int:
        """Primitive n-th root used by the reference tests (tests/fft.rs:16-24)."""
        log_n = int(math.floor(math.log2(n))) if n > 0 else 0
        w = self.two_adic_root()
        for _ in range(log_n, self.two_adicity):
            w = w * w % self.modulus
        return w


@dataclass(frozen=True)
class Curve:
    name: str
    fq: Field
    fr: Field
    b: int
    gx: int
    gy: int


BLS12_381_FR = Field(
    "bls12_381_fr",
    0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
    4, generator=7, two_adicity=32)
BLS12_381_FQ = Field(
    "bls12_381_fq",
    0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB,
    6)
BN254_FR = Field(
    "bn254_fr",
    0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,
    4, generator=5, two_adicity=28)
BN254_FQ = Field(
    "bn254_fq",
    0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,
    4)

BLS12_381 = Curve(
    "bls12_381", BLS12_381_FQ, BLS12_381_FR, 4,
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1)
BN254 = Curve("bn254", BN254_FQ, BN254_FR, 3, 1, 2)

FIELDS = {f.name: f for f in (BLS12_381_FR, BLS12_381_FQ, BN254_FR, BN254_FQ)}
CURVES = {c.name: c for c in (BLS12_381, BN254)}

# --------------------------------------------------------------------------
# Limb layout helpers: little-endian u64 limbs, the in-memory layout of
# ark_ff::BigInt<N> / Fp<MontBackend<_, N>, N> (ag-types/src/impls.rs:26-34)
# --------------------------------------------------------------------------


def int_to_limbs(x: int, n: int) -> list[int]:
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def limbs_to_int(limbs) -> int:
    return sum(int(v) << (64 * i) for i, v in enumerate(limbs))


# --------------------------------------------------------------------------
# FFT (ec-gpu-proxy/src/fft_cpu.rs) -- values are canonical ints mod r here;
# the Montgomery form only matters at the byte boundary.
# --------------------------------------------------------------------------


def pow_vartime(base: int, exp: int, mod: int) -> int:
    """ec-gpu-proxy/src/lib.rs:26-39 (square-and-multiply from the MSB)."""
    return pow(base, exp, mod)


def _bitreverse(n: int, l: int) -> int:
    r = 0
    for _ in range(l):
        r = (r << 1) | (n & 1)
        n >>= 1
    return r


def serial_fft(a: list[int], omega: int, log_n: int, mod: int) -> list[int]:
    """fft_cpu.rs:10-52: bit-reversal permutation then iterative radix-2 DIT."""
    a = list(a)
    n = len(a)
    assert n == 1 << log_n
    for k in range(n):
        rk = _bitreverse(k, log_n)
        if k < rk:
            a[k], a[rk] = a[rk], a[k]
    m = 1
    for _ in range(log_n):
        w_m = pow_vartime(omega, n // (2 * m), mod)
        k = 0
        while k < n:
            w = 1
            for j in range(m):
                t = a[k + j + m] * w % mod
                tmp = a[k + j]
                a[k + j + m] = (tmp - t) % mod
                a[k + j] = (tmp + t) % mod
                w = w * w_m % mod
            k += 2 * m
        m *= 2
    return a


def parallel_fft(a: list[int], omega: int, log_n: int, log_threads: int,
                 mod: int) -> list[int]:
    """fft_cpu.rs:59-111 (shuffle into 2^log_threads sub-FFTs + interleave)."""
    assert log_n >= log_threads
    num_threads = 1 << log_threads
    log_new_n = log_n - log_threads
    new_omega = pow_vartime(omega, num_threads, mod)
    tmp = []
    for j in range(num_threads):
        omega_j = pow_vartime(omega, j, mod)
        omega_step = pow_vartime(omega, j << log_new_n, mod)
        sub = [0] * (1 << log_new_n)
        elt = 1
        for i in range(1 << log_new_n):
            for s in range(num_threads):
                idx = (i + (s << log_new_n)) % (1 << log_n)
                sub[i] = (sub[i] + a[idx] * elt) % mod
                elt = elt * omega_step % mod
            elt = elt * omega_j % mod
        tmp.append(serial_fft(sub, new_omega, log_new_n, mod))
    mask = num_threads - 1
    return [tmp[idx & mask][idx >> log_threads] for idx in range(1 << log_n)]


def naive_dft(a: list[int], omega: int, mod: int) -> list[int]:
    n = len(a)
    return [sum(a[j] * pow(omega, j * k, mod) for j in range(n)) % mod
            for k in range(n)]


# --------------------------------------------------------------------------
# Short-Weierstrass Jacobian arithmetic over canonical ints, following the
# formula choice of ag-build/cl/ec.cl:17-120.  Identity = (0, 1, 0) (ec.cl:3).
# --------------------------------------------------------------------------

JAC_ZERO = (0, 1, 0)


def jac_double(P, p):
    """dbl-2009-l, ec.cl:17-42."""
    X, Y, Z = P
    if Z == 0:
        return P
    A = X * X % p
    B = Y * Y % p
    C = B * B % p
    D = 2 * (((X + B) ** 2) - A - C) % p
    E = 3 * A % p
    F = E * E % p
    Z3 = 2 * Y * Z % p
    X3 = (F - 2 * D) % p
    Y3 = (E * (D - X3) - 8 * C) % p
    return (X3, Y3, Z3)


def jac_add_mixed(P, Q, p):
    """madd-2007-bl, ec.cl:45-82 (Q affine (x, y); handles P == O and P == Q)."""
    X1, Y1, Z1 = P
    x2, y2 = Q
    if Z1 == 0:
        return (x2, y2, 1)
    Z1Z1 = Z1 * Z1 % p
    U2 = x2 * Z1Z1 % p
    S2 = y2 * Z1 * Z1Z1 % p
    if U2 == X1 and S2 == Y1:
        return jac_double(P, p)
    H = (U2 - X1) % p
    HH = H * H % p
    I = 4 * HH % p
    J = H * I % p
    r = 2 * (S2 - Y1) % p
    V = X1 * I % p
    X3 = (r * r - J - 2 * V) % p
    Y3 = (r * (V - X3) - 2 * Y1 * J) % p
    Z3 = ((Z1 + H) ** 2 - Z1Z1 - HH) % p
    return (X3, Y3, Z3)


def jac_add(P, Q, p):
    """add-2007-bl, ec.cl:85-120."""
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    if Z1 == 0:
        return Q
    if Z2 == 0:
        return P
    Z1Z1 = Z1 * Z1 % p
    Z2Z2 = Z2 * Z2 % p
    U1 = X1 * Z2Z2 % p
    U2 = X2 * Z1Z1 % p
    S1 = Y1 * Z2 * Z2Z2 % p
    S2 = Y2 * Z1 * Z1Z1 % p
    if U1 == U2 and S1 == S2:
        return jac_double(P, p)
    H = (U2 - U1) % p
    I = (2 * H) ** 2 % p
    J = H * I % p
    r = 2 * (S2 - S1) % p
    V = U1 * I % p
    X3 = (r * r - J - 2 * V) % p
    Y3 = (r * (V - X3) - 2 * S1 * J) % p
    Z3 = (((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H) % p
    return (X3, Y3, Z3)


def jac_to_affine(P, p):
    """Returns (x, y) or None for the identity."""
    X, Y, Z = P
    if Z == 0:
        return None
    zi = pow(Z, -1, p)
    zi2 = zi * zi % p
    return (X * zi2 % p, Y * zi2 * zi % p)


def jac_eq(P, Q, p) -> bool:
    return jac_to_affine(P, p) == jac_to_affine(Q, p)


def scalar_mul(P_aff, k: int, p: int):
    """Double-and-add from the MSB (ec.cl:136-148), affine input."""
    acc = JAC_ZERO
    for bit in bin(k)[2:] if k > 0 else "":
        acc = jac_double(acc, p)
        if bit == "1":
            acc = jac_add_mixed(acc, P_aff, p)
    return acc


# --------------------------------------------------------------------------
# multiexp_cpu (ec-gpu-proxy/src/multiexp_cpu.rs:244-367)
# --------------------------------------------------------------------------


class IdentityBaseError(ValueError):
    """multiexp_cpu.rs:57-61: 'Encountered an identity element in the CRS.'"""


def window_size_cpu(n: int) -> int:
    """multiexp_cpu.rs:353-357."""
    return 3 if n < 32 else int(math.ceil(math.log(float(n))))


def multiexp_cpu(curve: Curve, bases, exps, c: int | None = None):
    """bases: list of affine (x, y) canonical ints or None (identity).
    exps: canonical ints (BigInt<4> values).  Returns a Jacobian triple."""
    p = curve.fq.modulus
    if c is None:
        c = window_size_cpu(len(exps))
    nbits = curve.fr.bits

    def region(skip: int):
        acc = JAC_ZERO
        buckets = [JAC_ZERO] * ((1 << c) - 1)
        handle_trivial = skip == 0
        for base, exp in zip(bases, exps):
            if exp == 0:
                continue
            if exp == 1:
                if handle_trivial:
                    if base is None:
                        raise IdentityBaseError
                    acc = jac_add_mixed(acc, base, p)
                continue
            d = ((exp >> skip) & 0xFFFFFFFFFFFFFFFF) % (1 << c)
            if d != 0:
                if base is None:
                    raise IdentityBaseError
                buckets[d - 1] = jac_add_mixed(buckets[d - 1], base, p)
        running = JAC_ZERO
        for b in reversed(buckets):
            running = jac_add(running, b, p)
            acc = jac_add(acc, running, p)
        return acc

    parts = [region(skip) for skip in range(0, nbits, c)]
    acc = JAC_ZERO
    for part in reversed(parts):
        for _ in range(c):
            acc = jac_double(acc, p)
        acc = jac_add(acc, part, p)
    return acc


def naive_multiexp(curve: Curve, bases, exps):
    """multiexp_cpu.rs:385-399 (test_with_bls12's naive_multiexp)."""
    p = curve.fq.modulus
    acc = JAC_ZERO
    for b, e in zip(bases, exps):
        if b is None:
            continue
        acc = jac_add(acc, scalar_mul(b, e, p), p)
    return acc


def on_curve(curve: Curve, P) -> bool:
    x, y = P
    p = curve.fq.modulus
    return (y * y - x * x * x - curve.b) % p == 0


# --------------------------------------------------------------------------
# Deterministic input generation: xoshiro256** (seeded via splitmix64)
# --------------------------------------------------------------------------

M64 = 0xFFFFFFFFFFFFFFFF


class Xoshiro256ss:
    def __init__(self, seed: int):
        s = seed & M64
        self.s = []
        for _ in range(4):
            s = (s + 0x9E3779B97F4A7C15) & M64
            z = s
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            self.s.append(z ^ (z >> 31))

    @staticmethod
    def _rotl(x, k):
        return ((x << k) | (x >> (64 - k))) & M64

    def next(self) -> int:
        s = self.s
        result = (self._rotl((s[1] * 5) & M64, 7) * 9) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = self._rotl(s[3], 45)
        return result

    def field_element(self, f: Field) -> int:
        """Uniform in [0, modulus) by rejection on the top limb mask."""
        nbits = f.bits
        while True:
            v = 0
            for i in range(f.limbs64):
                v |= self.next() << (64 * i)
            v &= (1 << nbits) - 1
            if v < f.modulus:
                return v


# --------------------------------------------------------------------------
# Fq2 = Fq[u]/(u^2 + 1) (ag-build/cl/field2.cl:1-61; the quadratic extension
# of both BLS12-381 and BN254) and G2.  Fq2 overloads the int operators the
# formulas above use (+, -, *, **, % p, == 0, pow(z, -1, p)), so jac_double /
# jac_add / jac_add_mixed / multiexp_cpu run unchanged over Fq2.
# --------------------------------------------------------------------------


class Fq2:
    __slots__ = ("c0", "c1", "p")

    def __init__(self, c0: int, c1: int, p: int):
        self.c0, self.c1, self.p = c0 % p, c1 % p, p

    def _lift(self, o):
        return o if isinstance(o, Fq2) else Fq2(o, 0, self.p)

    def __add__(self, o):
        o = self._lift(o)
        return Fq2(self.c0 + o.c0, self.c1 + o.c1, self.p)

    __radd__ = __add__

    def __sub__(self, o):
        o = self._lift(o)
        return Fq2(self.c0 - o.c0, self.c1 - o.c1, self.p)

    def __rsub__(self, o):
        return self._lift(o) - self

    def __neg__(self):
        return Fq2(-self.c0, -self.c1, self.p)

    def __mul__(self, o):
        if isinstance(o, int):
            return Fq2(self.c0 * o, self.c1 * o, self.p)
        # (a0 + a1 u)(b0 + b1 u) = a0 b0 - a1 b1 + (a0 b1 + a1 b0) u  (field2.cl:34-47)
        return Fq2(self.c0 * o.c0 - self.c1 * o.c1, self.c0 * o.c1 + self.c1 * o.c0, self.p)

    __rmul__ = __mul__

    def __mod__(self, _p):
        return self

    def __pow__(self, e, mod=None):
        if e < 0:
            n = (self.c0 * self.c0 + self.c1 * self.c1) % self.p
            ni = pow(n, -1, self.p)
            return Fq2(self.c0 * ni, -self.c1 * ni, self.p) ** (-e)
        r = Fq2(1, 0, self.p)
        b = self
        while e:
            if e & 1:
                r = r * b
            b = b * b
            e >>= 1
        return r

    def __eq__(self, o):
        o = self._lift(o)
        return self.c0 == o.c0 and self.c1 == o.c1

    def __hash__(self):
        return hash((self.c0, self.c1))

    def __repr__(self):
        return f"Fq2({hex(self.c0)}, {hex(self.c1)})"


@dataclass(frozen=True)
class CurveG2:
    name: str
    fq: Field
    fr: Field
    b: tuple  # Fq2 coefficient (c0, c1)
    gx: tuple
    gy: tuple

    def fq2(self, c0: int, c1: int = 0) -> Fq2:
        return Fq2(c0, c1, self.fq.modulus)

    @property
    def gen(self):
        return (self.fq2(*self.gx), self.fq2(*self.gy))


# Public curve definitions: BLS12-381 G2 (y^2 = x^3 + 4(u + 1)), BN254 G2
# (y^2 = x^3 + 3/(9 + u), EIP-197 generator).  test_oracle_g2 checks on-curve
# and r * G2 = O for both before anything uses them.
BLS12_381_G2 = CurveG2(
    "bls12_381_g2", BLS12_381_FQ, BLS12_381_FR, (4, 4),
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE))
_bn_b2 = Fq2(3, 0, BN254_FQ.modulus) * (Fq2(9, 1, BN254_FQ.modulus) ** -1)
BN254_G2 = CurveG2(
    "bn254_g2", BN254_FQ, BN254_FR, (_bn_b2.c0, _bn_b2.c1),
    (10857046999023057135944570762232829481370756359578518086990519993285655852781,
     11559732032986387107991004021392285783925812861821192530917403151452391805634),
    (8495653923123431417604973247489272438418190587263600148770280649306958101930,
     4082367875863433681332203403145435568316851327593401208105741076214120093531))
CURVES_G2 = {c.name: c for c in (BLS12_381_G2, BN254_G2)}


def on_curve_g2(curve: CurveG2, P) -> bool:
    x, y = P
    return y * y - x * x * x - curve.fq2(*curve.b) == 0


def g2_scalar_mul(curve: CurveG2, P_aff, k: int):
    return scalar_mul(P_aff, k, curve.fq.modulus)


def g2_to_affine(curve: CurveG2, P):
    return jac_to_affine(P, curve.fq.modulus)


def g2_multiexp_cpu(curve: CurveG2, bases, exps, c: int | None = None):
    """multiexp_cpu over G2 (same restatement, Fq2 coordinates)."""
    return multiexp_cpu(curve, bases, exps, c)
