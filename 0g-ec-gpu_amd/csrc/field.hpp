// Prime-field arithmetic for gfx950 (CDNA4), Montgomery form with R = 2^(64 N)
// -- exactly ark_ff::Fp<MontBackend<_, N>, N>'s representation
// (ag-types/src/impls.rs:26-34), so device bytes == host arkworks bytes.
//
// Replaces the reference's dual-dialect field library ag-build/cl/field.cl
// (FIELD_add/sub/double/mul/pow/mont/unmont, :14-392) and the PTX carry-chain
// helpers in ag-build/cl/common.cl:47-248.  Design:
//
//  * Elements live in VGPRs as L = 2N little-endian u32 limbs.
//  * Multiplication is product-scanning ("FIPS") Montgomery: column k of
//    a*b and of m*p is accumulated into a 96-bit accumulator
//    (acc64 : top32).  Every 32x32 product is ONE v_mad_u64_u32 whose 64-bit
//    addend is the accumulator itself and whose carry-out (SGPR lane mask) is
//    folded into `top` by ONE v_addc_co_u32.  hipcc never emits this pair from
//    C++ (it rebuilds the 64-bit add from v_add_co/v_addc), so it is written as
//    inline asm: mad (half rate, 2 issue slots) + addc (1 slot) per product,
//    vs. mad + 3 adds for the __int128 formulation.
//  * Results are fully reduced (< p), so equality/zero tests are bytewise and
//    device outputs are bit-identical to the reference CPU path.
//  * All moduli used here leave >= 1 spare top bit, so a+b < 2^(32L) and the
//    single conditional subtraction suffices (field.cl:58-69 relies on it too).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ecg {

namespace params {
#include "params.inc"
}

#define ECG_DEV __device__ __forceinline__
#define ECG_HD __host__ __device__ __forceinline__

template <class P>
struct Fp {
  using Params = P;
  static constexpr int N = P::N;       // 64-bit limbs
  static constexpr int L = 2 * P::N;   // 32-bit limbs
  uint32_t v[L];

  static constexpr uint32_t p32(int i) {
    return (i & 1) ? (uint32_t)(P::P[i >> 1] >> 32) : (uint32_t)P::P[i >> 1];
  }
  static constexpr uint32_t one32(int i) {
    return (i & 1) ? (uint32_t)(P::ONE[i >> 1] >> 32) : (uint32_t)P::ONE[i >> 1];
  }
  static constexpr uint32_t r2_32(int i) {
    return (i & 1) ? (uint32_t)(P::R2[i >> 1] >> 32) : (uint32_t)P::R2[i >> 1];
  }
  static constexpr uint32_t inv32() { return (uint32_t)P::INV; }  // -p^-1 mod 2^32

  ECG_DEV static Fp zero() {
    Fp r;
#pragma unroll
    for (int i = 0; i < L; i++) r.v[i] = 0;
    return r;
  }
  ECG_DEV static Fp one() {
    Fp r;
#pragma unroll
    for (int i = 0; i < L; i++) r.v[i] = one32(i);
    return r;
  }
  ECG_DEV static Fp r2() {
    Fp r;
#pragma unroll
    for (int i = 0; i < L; i++) r.v[i] = r2_32(i);
    return r;
  }
};

// ---------------------------------------------------------------------------
// Carry-chain primitives
// ---------------------------------------------------------------------------

// The asm statements touch only their operands, so they are not volatile:
// the scheduler may then interleave independent products (measured: the
// 2^24 NTT runs 7% faster than with volatile, which pins program order).
// -DECG_ASM_QUAL=volatile restores the pinned form for A/B.
#ifndef ECG_ASM_QUAL
#define ECG_ASM_QUAL
#endif

// acc(96) += a * b   : v_mad_u64_u32 with carry-out + v_addc into top.
ECG_DEV void mac96(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm ECG_ASM_QUAL(
      "v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(top)
      : "v"(a), "v"(b));
}

// Same with b a wave-uniform (SGPR) operand (modulus limbs).
ECG_DEV void mac96s(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b_uniform) {
  uint64_t cc;
  asm ECG_ASM_QUAL(
      "v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(top)
      : "v"(a), "s"(b_uniform));
}

// Montgomery digit m = lo * (-p^-1) mod 2^32.  v_mul_lo_u32 is quarter rate on
// gfx950 (tools/mad_microbench.hip); the low half of a half-rate
// v_mad_u64_u32 with a zero addend is the same value at half the cost.
// (-p^-1 = 0xffffffff, BLS12-381 Fr: a plain negation.)
template <class P>
ECG_DEV uint32_t mont_digit(uint32_t lo) {
  constexpr uint32_t inv = (uint32_t)P::INV;
  if constexpr (inv == 0xffffffffu) {
    return 0u - lo;
  } else {
    uint64_t r, cc;
    asm ECG_ASM_QUAL("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cc) : "v"(lo), "s"(inv));
    return (uint32_t)r;
  }
}

// r = a + b over L limbs; returns carry-out.  __builtin_addc/subc lower to
// v_add_co_u32 / v_addc_co_u32 chains (one VALU op per limb).
template <int L>
ECG_DEV uint32_t add_limbs(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r[i] = __builtin_addc(a[i], b[i], c, &c);
  return c;
}

// r = a - b over L limbs; returns borrow (1) or 0.
template <int L>
ECG_DEV uint32_t sub_limbs(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r[i] = __builtin_subc(a[i], b[i], c, &c);
  return c;
}

// ---------------------------------------------------------------------------
// Field ops
// ---------------------------------------------------------------------------

// Conditional subtract p (input < 2p) -> fully reduced.
template <class P>
ECG_DEV void reduce_once(Fp<P>& a) {
  constexpr int L = Fp<P>::L;
  uint32_t t[L];
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) t[i] = __builtin_subc(a.v[i], Fp<P>::p32(i), c, &c);
  const bool borrow = c != 0;
#pragma unroll
  for (int i = 0; i < L; i++) a.v[i] = borrow ? a.v[i] : t[i];
}

template <class P>
ECG_DEV Fp<P> fadd(const Fp<P>& a, const Fp<P>& b) {
  Fp<P> r;
  add_limbs<Fp<P>::L>(r.v, a.v, b.v);  // no overflow: p < 2^(32L-1)
  reduce_once(r);
  return r;
}

template <class P>
ECG_DEV Fp<P> fdbl(const Fp<P>& a) { return fadd(a, a); }

template <class P>
ECG_DEV Fp<P> fsub(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  Fp<P> r;
  uint32_t borrow = sub_limbs<L>(r.v, a.v, b.v);
  // add p back if borrowed (masked add keeps the code branch-free)
  const uint32_t mask = 0u - borrow;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = __builtin_addc(r.v[i], Fp<P>::p32(i) & mask, c, &c);
  return r;
}

template <class P>
ECG_DEV Fp<P> fneg(const Fp<P>& a) {
  return fsub(Fp<P>::zero(), a);
}

template <class P>
ECG_DEV bool fis_zero(const Fp<P>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < Fp<P>::L; i++) o |= a.v[i];
  return o == 0;
}

template <class P>
ECG_DEV bool feq(const Fp<P>& a, const Fp<P>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < Fp<P>::L; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// Batched forms: K products per asm statement (hipcc pads one s_nop at every
// asm boundary; batching amortises it).  x*y with both operands in VGPRs:
#define ECG_MAC_STEP(X, Y)                         \
  "v_mad_u64_u32 %0, %1, " X ", " Y ", %0\n\t"     \
  "v_addc_co_u32 %2, %1, %2, 0, %1\n\t"
ECG_DEV void mac96x2(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  uint64_t cc;
  asm ECG_ASM_QUAL(ECG_MAC_STEP("%3", "%4") ECG_MAC_STEP("%5", "%6")
               : "+v"(acc), "=&s"(cc), "+v"(top)
               : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
ECG_DEV void mac96x3(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                     uint32_t a2, uint32_t b2) {
  uint64_t cc;
  asm ECG_ASM_QUAL(ECG_MAC_STEP("%3", "%4") ECG_MAC_STEP("%5", "%6") ECG_MAC_STEP("%7", "%8")
               : "+v"(acc), "=&s"(cc), "+v"(top)
               : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2));
}
ECG_DEV void mac96x4(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                     uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3) {
  uint64_t cc;
  asm ECG_ASM_QUAL(ECG_MAC_STEP("%3", "%4") ECG_MAC_STEP("%5", "%6") ECG_MAC_STEP("%7", "%8")
                   ECG_MAC_STEP("%9", "%10")
               : "+v"(acc), "=&s"(cc), "+v"(top)
               : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
}
// ... and with the second operand wave-uniform (modulus limbs in SGPRs).
ECG_DEV void mac96x2s(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  uint64_t cc;
  asm ECG_ASM_QUAL(ECG_MAC_STEP("%3", "%4") ECG_MAC_STEP("%5", "%6")
               : "+v"(acc), "=&s"(cc), "+v"(top)
               : "v"(a0), "s"(b0), "v"(a1), "s"(b1));
}
ECG_DEV void mac96x3s(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                      uint32_t a2, uint32_t b2) {
  uint64_t cc;
  asm ECG_ASM_QUAL(ECG_MAC_STEP("%3", "%4") ECG_MAC_STEP("%5", "%6") ECG_MAC_STEP("%7", "%8")
               : "+v"(acc), "=&s"(cc), "+v"(top)
               : "v"(a0), "s"(b0), "v"(a1), "s"(b1), "v"(a2), "s"(b2));
}
ECG_DEV void mac96x4s(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                      uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3) {
  uint64_t cc;
  asm ECG_ASM_QUAL(ECG_MAC_STEP("%3", "%4") ECG_MAC_STEP("%5", "%6") ECG_MAC_STEP("%7", "%8")
                   ECG_MAC_STEP("%9", "%10")
               : "+v"(acc), "=&s"(cc), "+v"(top)
               : "v"(a0), "s"(b0), "v"(a1), "s"(b1), "v"(a2), "s"(b2), "v"(a3), "s"(b3));
}
#undef ECG_MAC_STEP

// acc(96) += sum_{t<CNT} x[t]*y[t]; UNIFORM selects SGPR operands for y.
template <int CNT, bool UNIFORM>
ECG_DEV void mac_list(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) {
  int t = 0;
#pragma unroll
  for (; t + 4 <= CNT; t += 4) {
    if (UNIFORM) mac96x4s(acc, top, x[t], y[t], x[t + 1], y[t + 1], x[t + 2], y[t + 2], x[t + 3], y[t + 3]);
    else mac96x4(acc, top, x[t], y[t], x[t + 1], y[t + 1], x[t + 2], y[t + 2], x[t + 3], y[t + 3]);
  }
  constexpr int REM = CNT % 4;
  constexpr int T0 = CNT - REM;
  if (REM == 3) {
    if (UNIFORM) mac96x3s(acc, top, x[T0], y[T0], x[T0 + 1], y[T0 + 1], x[T0 + 2], y[T0 + 2]);
    else mac96x3(acc, top, x[T0], y[T0], x[T0 + 1], y[T0 + 1], x[T0 + 2], y[T0 + 2]);
  } else if (REM == 2) {
    if (UNIFORM) mac96x2s(acc, top, x[T0], y[T0], x[T0 + 1], y[T0 + 1]);
    else mac96x2(acc, top, x[T0], y[T0], x[T0 + 1], y[T0 + 1]);
  } else if (REM == 1) {
    if (UNIFORM) mac96s(acc, top, x[T0], y[T0]);
    else mac96(acc, top, x[T0], y[T0]);
  }
}

// One column of the product-scanning Montgomery product (k < L: reduction
// digit m[k] produced; k >= L: output limb r[k-L]).
template <class P, int K>
ECG_DEV void fmul_column(uint64_t& acc, uint32_t& top, const uint32_t* a, const uint32_t* b, uint32_t* m,
                         uint32_t* r) {
  constexpr int L = Fp<P>::L;
  constexpr int I0 = K < L ? 0 : K - L + 1;
  constexpr int I1 = K < L ? K : L - 1;  // inclusive, ab part
  constexpr int NAB = I1 - I0 + 1;
  constexpr int NMP = K < L ? K : L - I0;  // m[i]*p[K-i], i in [I0, min(K, L)-1]
  uint32_t xs[NAB], ys[NAB];
#pragma unroll
  for (int t = 0; t < NAB; t++) { xs[t] = a[I0 + t]; ys[t] = b[K - I0 - t]; }
  mac_list<NAB, false>(acc, top, xs, ys);
  if constexpr (NMP > 0) {
    uint32_t xm[NMP], pm[NMP];
#pragma unroll
    for (int t = 0; t < NMP; t++) { xm[t] = m[I0 + t]; pm[t] = Fp<P>::p32(K - I0 - t); }
    mac_list<NMP, true>(acc, top, xm, pm);
  }
  if constexpr (K < L) {
    m[K] = mont_digit<P>((uint32_t)acc);
    mac96s(acc, top, m[K], Fp<P>::p32(0));  // low word of acc becomes 0
  } else {
    r[K - L] = (uint32_t)acc;
  }
  acc = (acc >> 32) | ((uint64_t)top << 32);
  top = 0;
}

template <class P, int K>
ECG_DEV void fmul_columns(uint64_t& acc, uint32_t& top, const uint32_t* a, const uint32_t* b, uint32_t* m,
                          uint32_t* r) {
  if constexpr (K < 2 * Fp<P>::L - 1) {
    fmul_column<P, K>(acc, top, a, b, m, r);
    fmul_columns<P, K + 1>(acc, top, a, b, m, r);
  }
}

// Batched-asm variant (4 products per asm statement).  Measured slower than
// the unbatched form on gfx950 (Fr 115.4 vs 128.7 G mul/s, tools/field_bench):
// coarse asm blocks stop hipcc interleaving independent multiplications.
template <class P>
ECG_DEV Fp<P> fmul_x4(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  uint32_t m[L];
  Fp<P> r;
  uint64_t acc = 0;
  uint32_t top = 0;
  fmul_columns<P, 0>(acc, top, a.v, b.v, m, r.v);
  r.v[L - 1] = (uint32_t)acc;  // result < 2p < 2^(32L): acc >> 32 == 0 here
  reduce_once(r);
  return r;
}

// Montgomery product a*b*R^-1 mod p, product-scanning (FIPS) form, one
// product per asm statement (the default: fastest measured form).
// REDUCE = false skips the final conditional subtraction (lazy form, below).
template <class P, bool REDUCE = true>
ECG_DEV Fp<P> fmul(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  uint32_t m[L];
  Fp<P> r;
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < L; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) mac96(acc, top, a.v[i], b.v[k - i]);
#pragma unroll
    for (int i = 0; i < k; i++) mac96s(acc, top, m[i], Fp<P>::p32(k - i));
    m[k] = mont_digit<P>((uint32_t)acc);
    mac96s(acc, top, m[k], Fp<P>::p32(0));
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
#pragma unroll
  for (int k = L; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = k - L + 1; i < L; i++) mac96(acc, top, a.v[i], b.v[k - i]);
#pragma unroll
    for (int i = k - L + 1; i < L; i++) mac96s(acc, top, m[i], Fp<P>::p32(k - i));
    r.v[k - L] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  r.v[L - 1] = (uint32_t)acc;
  if constexpr (REDUCE) reduce_once(r);
  return r;
}

// Two-chain form (A/B variant): each column's a*b and m*p products accumulate
// in two independent 96-bit chains merged before the Montgomery digit.
// Measured ~12% SLOWER than fmul at every occupancy, 1..8 waves/SIMD
// (profiles/r01/field_bench_ilp2.log): the product is issue-bound on
// v_mad_u64_u32 + v_addc, not latency-bound, so extra merge ops only cost.
ECG_DEV void add96(uint64_t& acc, uint32_t& top, uint64_t acc2, uint32_t top2) {
  const uint64_t s = acc + acc2;
  top += top2 + (s < acc ? 1u : 0u);
  acc = s;
}

template <class P, bool REDUCE = true>
ECG_DEV Fp<P> fmul_ilp(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  uint32_t m[L];
  Fp<P> r;
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < L; k++) {
    uint64_t acc2 = 0;
    uint32_t top2 = 0;
#pragma unroll
    for (int i = 0; i <= k; i++) {
      mac96(acc, top, a.v[i], b.v[k - i]);
      if (i < k) mac96s(acc2, top2, m[i], Fp<P>::p32(k - i));
    }
    add96(acc, top, acc2, top2);
    m[k] = mont_digit<P>((uint32_t)acc);
    mac96s(acc, top, m[k], Fp<P>::p32(0));
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
#pragma unroll
  for (int k = L; k < 2 * L - 1; k++) {
    uint64_t acc2 = 0;
    uint32_t top2 = 0;
#pragma unroll
    for (int i = k - L + 1; i < L; i++) {
      mac96(acc, top, a.v[i], b.v[k - i]);
      mac96s(acc2, top2, m[i], Fp<P>::p32(k - i));
    }
    add96(acc, top, acc2, top2);
    r.v[k - L] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  r.v[L - 1] = (uint32_t)acc;
  if constexpr (REDUCE) reduce_once(r);
  return r;
}

template <class P>
ECG_DEV Fp<P> fsqr(const Fp<P>& a) { return fmul(a, a); }

// ---------------------------------------------------------------------------
// Lazy ("redundant") arithmetic for moduli with 4p < 2^(32L): values live in
// [0, 2p].  Closed under Montgomery multiplication with NO final subtraction
// (a, b <= 2p  =>  (ab + mp)/R < 4p^2/R + p < 2p), and add/sub/neg each need
// one correction by 2p.  Used by the MSM bucket arithmetic over both base
// fields; every value that leaves the MSM pipeline is canonicalised first
// (freduce_full), so outputs stay bit-identical to the reference's.
// ---------------------------------------------------------------------------
template <class P>
struct Lazy {
  static constexpr bool ok() { return (P::P[P::N - 1] >> 62) == 0; }  // p < 2^(64N-2)  <=>  4p < R
};

// 2p as 32-bit limbs (carry of the 64-bit shift handled explicitly)
template <class P>
ECG_DEV constexpr uint32_t p2_limb(int i) {
  const int w = i >> 1;
  const uint64_t lo = P::P[w] << 1 | (w > 0 ? P::P[w - 1] >> 63 : 0);
  return (i & 1) ? (uint32_t)(lo >> 32) : (uint32_t)lo;
}

template <class P>
ECG_DEV Fp<P> fmul_lz(const Fp<P>& a, const Fp<P>& b) {
  static_assert(Lazy<P>::ok(), "lazy reduction needs 4p < R");
  return fmul<P, false>(a, b);
}

template <class P>
ECG_DEV Fp<P> fsqr_lz(const Fp<P>& a) { return fmul_lz(a, a); }

// a + b with a, b in [0, 2p] -> [0, 2p]
template <class P>
ECG_DEV Fp<P> fadd_lz(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  Fp<P> r;
  uint32_t t[L];
  add_limbs<L>(r.v, a.v, b.v);  // < 4p < R: no carry-out
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) t[i] = __builtin_subc(r.v[i], p2_limb<P>(i), c, &c);
  const bool borrow = c != 0;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = borrow ? r.v[i] : t[i];
  return r;
}

template <class P>
ECG_DEV Fp<P> fdbl_lz(const Fp<P>& a) { return fadd_lz(a, a); }

// a - b with a, b in [0, 2p] -> [0, 2p]
template <class P>
ECG_DEV Fp<P> fsub_lz(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  Fp<P> r;
  const uint32_t borrow = sub_limbs<L>(r.v, a.v, b.v);
  const uint32_t mask = 0u - borrow;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = __builtin_addc(r.v[i], p2_limb<P>(i) & mask, c, &c);
  return r;
}

// 2p - a, a in [0, 2p] -> [0, 2p]: one subtraction, no correction
template <class P>
ECG_DEV Fp<P> fneg_lz(const Fp<P>& a) {
  constexpr int L = Fp<P>::L;
  Fp<P> r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = __builtin_subc(p2_limb<P>(i), a.v[i], c, &c);
  return r;
}

// [0, 2p] -> canonical [0, p)
template <class P>
ECG_DEV Fp<P> freduce_full(Fp<P> a) {
  reduce_once(a);  // [0, 2p] -> [0, p]
  reduce_once(a);  // p -> 0
  return a;
}

// a == 0 (mod p) for a in [0, 2p]
template <class P>
ECG_DEV bool fis_zero_lz(const Fp<P>& a) {
  constexpr int L = Fp<P>::L;
  uint32_t z = 0, e1 = 0, e2 = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    z |= a.v[i];
    e1 |= a.v[i] ^ Fp<P>::p32(i);
    e2 |= a.v[i] ^ p2_limb<P>(i);
  }
  return z == 0 || e1 == 0 || e2 == 0;
}

// Portable CIOS reference variant (row-wise u64 chains) -- kept for A/B
// measurement against the asm product-scanning form (tools/field_bench).
template <class P>
ECG_DEV Fp<P> fmul_cios(const Fp<P>& a, const Fp<P>& b) {
  constexpr int L = Fp<P>::L;
  uint32_t t[L + 2];
#pragma unroll
  for (int i = 0; i < L + 2; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; j++) {
      uint64_t x = (uint64_t)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint32_t)x;
      c = (uint32_t)(x >> 32);
    }
    uint64_t x = (uint64_t)t[L] + c;
    t[L] = (uint32_t)x;
    t[L + 1] = (uint32_t)(x >> 32);
    uint32_t mm = t[0] * Fp<P>::inv32();
    x = (uint64_t)mm * Fp<P>::p32(0) + t[0];
    c = (uint32_t)(x >> 32);
#pragma unroll
    for (int j = 1; j < L; j++) {
      x = (uint64_t)mm * Fp<P>::p32(j) + t[j] + c;
      t[j - 1] = (uint32_t)x;
      c = (uint32_t)(x >> 32);
    }
    x = (uint64_t)t[L] + c;
    t[L - 1] = (uint32_t)x;
    t[L] = t[L + 1] + (uint32_t)(x >> 32);
  }
  Fp<P> r;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = t[i];
  reduce_once(r);
  return r;
}

// a^e for a small exponent (square-and-multiply, LSB first) -- field.cl:329-338
template <class P>
ECG_DEV Fp<P> fpow_u32(Fp<P> base, uint32_t e) {
  Fp<P> r = Fp<P>::one();
  while (e) {
    if (e & 1) r = fmul(r, base);
    e >>= 1;
    if (e) base = fsqr(base);
  }
  return r;
}

// a^(p-2) (Fermat inverse); a == 0 -> 0.
template <class P>
ECG_DEV Fp<P> finv(const Fp<P>& a) {
  Fp<P> r = Fp<P>::one();
  for (int i = P::N - 1; i >= 0; i--) {
    uint64_t e = P::PM2[i];
    for (int bit = 63; bit >= 0; bit--) {
      r = fsqr(r);
      if ((e >> bit) & 1) r = fmul(r, a);
    }
  }
  return r;
}

// Montgomery <-> canonical (field.cl:355-377)
template <class P>
ECG_DEV Fp<P> to_mont(const Fp<P>& a) { return fmul(a, Fp<P>::r2()); }
template <class P>
ECG_DEV Fp<P> from_mont(const Fp<P>& a) {
  Fp<P> one = Fp<P>::zero();
  one.v[0] = 1;
  return fmul(a, one);
}

// Global-memory load/store of one element as 16-byte vectors.
template <class P>
ECG_DEV Fp<P> load(const Fp<P>* p) {
  Fp<P> r;
  const uint4* s = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < Fp<P>::L / 4; i++) {
    uint4 q = s[i];
    r.v[4 * i] = q.x; r.v[4 * i + 1] = q.y; r.v[4 * i + 2] = q.z; r.v[4 * i + 3] = q.w;
  }
  return r;
}
template <class P>
ECG_DEV void store(Fp<P>* p, const Fp<P>& a) {
  uint4* d = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < Fp<P>::L / 4; i++)
    d[i] = make_uint4(a.v[4 * i], a.v[4 * i + 1], a.v[4 * i + 2], a.v[4 * i + 3]);
}

using FrBLS = Fp<params::bls12_381_fr>;
using FqBLS = Fp<params::bls12_381_fq>;
using FrBN = Fp<params::bn254_fr>;
using FqBN = Fp<params::bn254_fq>;

}  // namespace ecg
