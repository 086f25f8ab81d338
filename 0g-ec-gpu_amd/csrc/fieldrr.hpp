// Reduced-radix Montgomery arithmetic for the MSM bucket pipeline (gfx950).
//
// field.hpp's 32-bit-limb product needs a v_addc_co_u32 after every
// v_mad_u64_u32 to catch the 64-bit accumulator's carry, and on gfx950 that
// addc issues at the same cost as the mad itself (tools/issue_bench.hip:
// mad, addc, add_co, mul_lo, alignbit all ~4 SIMD cycles per wave64; only
// v_add_u32 is cheaper).  Here an element is NL limbs of BITS <= 29 bits:
// every product is < 2^58, a whole column of 2*NL products fits a plain
// 64-bit accumulator, and a product is ONE v_mad_u64_u32.  One shift per
// column replaces the 2*L^2 carry instructions: the BLS12-381 Fq product
// drops from ~640 to ~470 VALU instructions.
//
// Representation  FpR<Q>: value = sum v[i] 2^(BITS i) = x R' (mod p), with
// R' = 2^(NL BITS) (Q = params::*_rr, tools/gen_params_rr.py).  The boundary
// keeps ark-ff's R = 2^(64N) form; rr_from_std / rr_to_std convert (one
// product each).  Values are redundant ("lazy"):
//   * quasi-normalised (QN): limbs i < NL-1 below 2^BITS + 8, top limb holds
//     the rest of the value;
//   * rr_mul / rr_sqr: QN inputs of values a, b with a*b <= 2^SLACK_LOG2 p^2 / 2
//     -> output (ab + mp)/R' < p + p/2, with EXACT limbs (< 2^BITS), so the
//     output is the unique radix-2^BITS digit string of its value;
//   * rr_add: exact sum, QN;  rr_sub<k>: a - b + k p, QN, for b <= k p / 2;
//   * congruence to 0 of a product output v (< 2p) is  v == 0 || v == p.
// The MSM formulas (curve_rr.hpp) keep every value below 64 p, far inside
// the 2^25 (BLS12-381 Fq) / 2^26 (BN254 Fq) slack.  Outputs are converted back
// and fully reduced, so results stay bit-identical to the reference's.
#pragma once
#include "field.hpp"

namespace ecg {

namespace params {
#include "params_rr.inc"
}

template <class Q>
struct FpR {
  using Params = Q;
  static constexpr int NL = Q::NL;
  static constexpr int B = Q::BITS;
  static constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t v[NL];

  ECG_DEV static FpR zero() {
    FpR r;
#pragma unroll
    for (int i = 0; i < NL; i++) r.v[i] = 0;
    return r;
  }
  ECG_DEV static FpR one() {
    FpR r;
#pragma unroll
    for (int i = 0; i < NL; i++) r.v[i] = Q::ONE[i];
    return r;
  }
};

// acc += a * b as ONE v_mad_u64_u32 (carry-out unused: the column sum never
// exceeds 2^63).  Written as asm so that hipcc keeps one accumulator chain per
// column instead of re-associating it into two chains joined by a 64-bit add
// (measured: that costs ~8% more instructions per product).
ECG_DEV void mad64(uint64_t& acc, uint32_t a, uint32_t b) {
#if defined(ECG_RR_CXX_MAD)
  acc += (uint64_t)a * b;
#elif defined(ECG_RR_BAR_MAD)
  acc += (uint64_t)a * b;
  asm("" : "+v"(acc));
#else
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
#endif
}
ECG_DEV void mad64s(uint64_t& acc, uint32_t a, uint32_t b_uniform) {
#if defined(ECG_RR_CXX_MAD)
  acc += (uint64_t)a * b_uniform;
#elif defined(ECG_RR_BAR_MAD)
  acc += (uint64_t)a * b_uniform;
  asm("" : "+v"(acc));
#else
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "s"(b_uniform));
#endif
}

// Montgomery product (a b + m p) / R', product scanning, one v_mad_u64_u32
// per product.
// Moduli with P[0] = 1 (BLS12-381 Fr: r = 1 mod 2^32).  The digit m = -x mod
// 2^B makes x + m the next multiple of 2^B, so the column carry is ceil(x /
// 2^B) and the m P[0] mad is not needed.  The chains carry z = x - 1 instead
// (column 0 starts at -1): ceil(x / 2^B) = (z >> B) + 1 with an arithmetic
// shift, m = ~z mod 2^B, and the +1 of one column cancels the -1 of the next,
// so only the last reduction column adds it back.  9 mads fewer per Fr
// product; columns stay below 2^63 in magnitude, so z never wraps.
template <class Q>
constexpr bool rr_ceil_carry() {
  return Q::P[0] == 1;
}
template <class Q>
ECG_DEV void rr_ceil_step(uint64_t& z, uint32_t& m, bool last) {
  constexpr uint32_t MASK = (1u << Q::BITS) - 1;
  m = ~(uint32_t)z & MASK;
  z = (uint64_t)((int64_t)z >> Q::BITS);
  if (last) z += 1;
}

// Column splits (BITS = 30: BLS12-381's 13 x 30-bit G1 layout).  A product
// of two QN limbs (<= 2^30 + 3) is just above 2^60, so a 64-bit column holds
// about 15 of them.  The m p products of a column are bounded by the modulus
// limbs themselves (sum of (2^30 - 1) P_j over the column's j, at most 6.7
// x 2^60 for all 13 limbs), so only the columns whose bound below -- `sets`
// NL-product sets of QN limbs (a b; a b + c d in rr_mul_sum2), the m p terms
// and a 2^37 carry-in -- reaches 2^64 are split (columns 10-14 of a 13-limb
// product): after the a b products the accumulator keeps its low BITS bits
// and the rest (h, a multiple of 2^BITS) skips the m p products and rejoins
// the carry-out.  A squaring's doubled off-diagonal product counts twice, so
// its columns bound like a product's.  BITS <= 29 never splits (2 NL
// products of 2^58 fit).
template <class Q>
constexpr int rr_col_half(int k) {  // a b (or m p) products in column k
  return k < Q::NL ? k + 1 : 2 * Q::NL - 1 - k;
}
template <class Q>
constexpr bool rr_col_fits(int k, int sets) {
  using u128 = unsigned __int128;
  const u128 lim = (u128)1 << Q::BITS, qn = lim + 3;
  u128 s = (u128)sets * (u128)rr_col_half<Q>(k) * qn * qn + ((u128)1 << 37);
  const int j0 = k < Q::NL ? 0 : k - Q::NL + 1, j1 = k < Q::NL ? k : Q::NL - 1;
  for (int j = j0; j <= j1; j++) s += (lim - 1) * (u128)Q::P[j];
  return s < ((u128)1 << 64);
}
template <class Q>
constexpr bool rr_col_split(int k, int sets = 1) {
  return Q::BITS > 29 && !rr_col_fits<Q>(k, sets);
}
// (Keeping the low 32 bits instead -- h = the high word, no shift -- costs
// more: the zeroed high word and the joined h need 64-bit moves.)
template <class Q>
ECG_DEV void rr_split(uint64_t& x, uint64_t& h) {
  static_assert(Q::BITS <= 29 || !rr_ceil_carry<Q>(), "the ceil-carry chains (signed z) are not split");
  h = x >> Q::BITS;
  x &= (uint64_t)((1u << Q::BITS) - 1);
}
template <class Q>
ECG_DEV void rr_join(uint64_t& x, uint64_t h) {
  x += h;
}

// Montgomery product (a b + m p) / R', product scanning, one v_mad_u64_u32
// per product.
template <class Q>
ECG_DEV FpR<Q> rr_mul(const FpR<Q>& a, const FpR<Q>& b) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m[NL];
  FpR<Q> r;
  uint64_t acc = rr_ceil_carry<Q>() ? ~0ull : 0ull;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) mad64(acc, a.v[i], b.v[k - i]);
    uint64_t h = 0;
    if (rr_col_split<Q>(k)) rr_split<Q>(acc, h);
#pragma unroll
    for (int i = 0; i < k; i++) mad64s(acc, m[i], Q::P[k - i]);
    if constexpr (rr_ceil_carry<Q>()) {
      rr_ceil_step<Q>(acc, m[k], k == NL - 1);
    } else {
      m[k] = ((uint32_t)acc * Q::INV) & MASK;
      mad64s(acc, m[k], Q::P[0]);  // low BITS bits of acc become 0
      acc >>= B;
      if (rr_col_split<Q>(k)) rr_join<Q>(acc, h);
    }
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) mad64(acc, a.v[i], b.v[k - i]);
    uint64_t h = 0;
    if (rr_col_split<Q>(k)) rr_split<Q>(acc, h);
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) mad64s(acc, m[i], Q::P[k - i]);
    r.v[k - NL] = (uint32_t)acc & MASK;
    acc >>= B;
    if (rr_col_split<Q>(k)) rr_join<Q>(acc, h);
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// Two independent products column by column, their mads paired in one asm
// statement: two dependency chains in flight per wave (latency cover at 2
// waves/SIMD) and one hazard s_nop per pair instead of per product.
ECG_DEV void mad64x2(uint64_t& acc0, uint32_t a0, uint32_t b0, uint64_t& acc1, uint32_t a1, uint32_t b1) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_mad_u64_u32 %1, %3, %6, %7, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(c0), "=&s"(c1)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
ECG_DEV void mad64x2s(uint64_t& acc0, uint32_t a0, uint64_t& acc1, uint32_t a1, uint32_t b_uniform) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %2, %4, %6, %0\n\t"
      "v_mad_u64_u32 %1, %3, %5, %6, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(c0), "=&s"(c1)
      : "v"(a0), "v"(a1), "s"(b_uniform));
}

// Four mads -- two per chain -- per asm statement: half the statement
// boundaries, after each of which the compiler places a hazard s_nop
// (A/B: -DECG_RR_NO_X4 keeps two mads per statement).
ECG_DEV void mad64x4(uint64_t& acc0, uint32_t a0, uint32_t b0, uint32_t c0, uint32_t d0, uint64_t& acc1, uint32_t a1,
                     uint32_t b1, uint32_t c1, uint32_t d1) {
  uint64_t k0, k1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_mad_u64_u32 %1, %3, %8, %9, %1\n\t"
      "v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
      "v_mad_u64_u32 %1, %3, %10, %11, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(k0), "=&s"(k1)
      : "v"(a0), "v"(b0), "v"(c0), "v"(d0), "v"(a1), "v"(b1), "v"(c1), "v"(d1));
}
// acc0 += a0 u + c0 w, acc1 += a1 u + c1 w  (u, w uniform)
ECG_DEV void mad64x4s(uint64_t& acc0, uint32_t a0, uint32_t c0, uint64_t& acc1, uint32_t a1, uint32_t c1, uint32_t u,
                      uint32_t w) {
  uint64_t k0, k1;
  asm("v_mad_u64_u32 %0, %2, %4, %8, %0\n\t"
      "v_mad_u64_u32 %1, %3, %6, %8, %1\n\t"
      "v_mad_u64_u32 %0, %2, %5, %9, %0\n\t"
      "v_mad_u64_u32 %1, %3, %7, %9, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(k0), "=&s"(k1)
      : "v"(a0), "v"(c0), "v"(a1), "v"(c1), "s"(u), "s"(w));
}

// Eight mads -- four per chain -- per asm statement (A/B: -DECG_RR_X4_ONLY).
ECG_DEV void mad64x8(uint64_t& acc0, const uint32_t* a0, const uint32_t* b0, uint64_t& acc1, const uint32_t* a1,
                     const uint32_t* b1) {
  uint64_t k0, k1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_mad_u64_u32 %1, %3, %12, %13, %1\n\t"
      "v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
      "v_mad_u64_u32 %1, %3, %14, %15, %1\n\t"
      "v_mad_u64_u32 %0, %2, %8, %9, %0\n\t"
      "v_mad_u64_u32 %1, %3, %16, %17, %1\n\t"
      "v_mad_u64_u32 %0, %2, %10, %11, %0\n\t"
      "v_mad_u64_u32 %1, %3, %18, %19, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(k0), "=&s"(k1)
      : "v"(a0[0]), "v"(b0[0]), "v"(a0[1]), "v"(b0[1]), "v"(a0[2]), "v"(b0[2]), "v"(a0[3]), "v"(b0[3]),
        "v"(a1[0]), "v"(b1[0]), "v"(a1[1]), "v"(b1[1]), "v"(a1[2]), "v"(b1[2]), "v"(a1[3]), "v"(b1[3]));
}
// acc0 += sum_t m0[t] u[t], acc1 += sum_t m1[t] u[t], t < 4 (u uniform)
ECG_DEV void mad64x8s(uint64_t& acc0, const uint32_t* m0, uint64_t& acc1, const uint32_t* m1, const uint32_t* u) {
  uint64_t k0, k1;
  asm("v_mad_u64_u32 %0, %2, %4, %12, %0\n\t"
      "v_mad_u64_u32 %1, %3, %8, %12, %1\n\t"
      "v_mad_u64_u32 %0, %2, %5, %13, %0\n\t"
      "v_mad_u64_u32 %1, %3, %9, %13, %1\n\t"
      "v_mad_u64_u32 %0, %2, %6, %14, %0\n\t"
      "v_mad_u64_u32 %1, %3, %10, %14, %1\n\t"
      "v_mad_u64_u32 %0, %2, %7, %15, %0\n\t"
      "v_mad_u64_u32 %1, %3, %11, %15, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(k0), "=&s"(k1)
      : "v"(m0[0]), "v"(m0[1]), "v"(m0[2]), "v"(m0[3]), "v"(m1[0]), "v"(m1[1]), "v"(m1[2]), "v"(m1[3]),
        "s"(u[0]), "s"(u[1]), "s"(u[2]), "s"(u[3]));
}

// First products of a column: the same pairs with a zero addend for chain 0
// (Z0) and/or chain 1 (Z1), which starts that accumulator instead of a
// v_mov_b64 of 0 ahead of the column.
template <bool Z0, bool Z1>
ECG_DEV void mad64x2_z(uint64_t& acc0, uint32_t a0, uint32_t b0, uint64_t& acc1, uint32_t a1, uint32_t b1) {
  uint64_t c0, c1;
  if constexpr (Z0 && Z1)
    asm("v_mad_u64_u32 %0, %2, %4, %5, 0\n\t"
        "v_mad_u64_u32 %1, %3, %6, %7, 0"
        : "=&v"(acc0), "=&v"(acc1), "=&s"(c0), "=&s"(c1)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
  else if constexpr (Z1)
    asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
        "v_mad_u64_u32 %1, %3, %6, %7, 0"
        : "+v"(acc0), "=&v"(acc1), "=&s"(c0), "=&s"(c1)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
  else
    mad64x2(acc0, a0, b0, acc1, a1, b1);
}
// First products of both chains with an addend of -1 (rr_ceil_carry's z form).
ECG_DEV void mad64x2_m1(uint64_t& acc0, uint32_t a0, uint32_t b0, uint64_t& acc1, uint32_t a1, uint32_t b1) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, -1\n\t"
      "v_mad_u64_u32 %1, %3, %6, %7, -1"
      : "=&v"(acc0), "=&v"(acc1), "=&s"(c0), "=&s"(c1)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
// acc0 += a0 b0 + c0 d0; acc1 = a1 b1 + c1 d1 (chain 1 starts at zero)
ECG_DEV void mad64x4_z1(uint64_t& acc0, uint32_t a0, uint32_t b0, uint32_t c0, uint32_t d0, uint64_t& acc1,
                        uint32_t a1, uint32_t b1, uint32_t c1, uint32_t d1) {
  uint64_t k0, k1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_mad_u64_u32 %1, %3, %8, %9, 0\n\t"
      "v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
      "v_mad_u64_u32 %1, %3, %10, %11, %1"
      : "+v"(acc0), "=&v"(acc1), "=&s"(k0), "=&s"(k1)
      : "v"(a0), "v"(b0), "v"(c0), "v"(d0), "v"(a1), "v"(b1), "v"(c1), "v"(d1));
}
// mad64x8 with chain 1 starting at zero
ECG_DEV void mad64x8_z1(uint64_t& acc0, const uint32_t* a0, const uint32_t* b0, uint64_t& acc1, const uint32_t* a1,
                        const uint32_t* b1) {
  uint64_t k0, k1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_mad_u64_u32 %1, %3, %12, %13, 0\n\t"
      "v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
      "v_mad_u64_u32 %1, %3, %14, %15, %1\n\t"
      "v_mad_u64_u32 %0, %2, %8, %9, %0\n\t"
      "v_mad_u64_u32 %1, %3, %16, %17, %1\n\t"
      "v_mad_u64_u32 %0, %2, %10, %11, %0\n\t"
      "v_mad_u64_u32 %1, %3, %18, %19, %1"
      : "+v"(acc0), "=&v"(acc1), "=&s"(k0), "=&s"(k1)
      : "v"(a0[0]), "v"(b0[0]), "v"(a0[1]), "v"(b0[1]), "v"(a0[2]), "v"(b0[2]), "v"(a0[3]), "v"(b0[3]),
        "v"(a1[0]), "v"(b1[0]), "v"(a1[1]), "v"(b1[1]), "v"(a1[2]), "v"(b1[2]), "v"(a1[3]), "v"(b1[3]));
}

// Column pieces of two interleaved products (k, lo, hi fold to constants in
// the unrolled column loops): sum_{lo <= i <= hi} a_i b_{k-i} into (x0, x1),
// and sum_{lo <= i <= hi} m_i P_{k-i} for the uniform modulus limbs P.
// Z1: chain 1 starts at zero with the column's first statement (lo <= hi).
template <bool Z1 = false>
ECG_DEV void col2(int k, int lo, int hi, uint64_t& x0, const uint32_t* a0, const uint32_t* b0, uint64_t& x1,
                  const uint32_t* a1, const uint32_t* b1) {
  bool first = Z1;
#if !defined(ECG_RR_NO_X4) && !defined(ECG_RR_X4_ONLY)
  for (; lo + 3 <= hi; lo += 4) {
    const uint32_t ta0[4] = {a0[lo], a0[lo + 1], a0[lo + 2], a0[lo + 3]};
    const uint32_t tb0[4] = {b0[k - lo], b0[k - lo - 1], b0[k - lo - 2], b0[k - lo - 3]};
    const uint32_t ta1[4] = {a1[lo], a1[lo + 1], a1[lo + 2], a1[lo + 3]};
    const uint32_t tb1[4] = {b1[k - lo], b1[k - lo - 1], b1[k - lo - 2], b1[k - lo - 3]};
    if (first)
      mad64x8_z1(x0, ta0, tb0, x1, ta1, tb1);
    else
      mad64x8(x0, ta0, tb0, x1, ta1, tb1);
    first = false;
  }
#endif
#pragma unroll
  for (int i = lo; i <= hi; i += 2) {
#ifndef ECG_RR_NO_X4
    if (i + 1 <= hi) {
      if (first)
        mad64x4_z1(x0, a0[i], b0[k - i], a0[i + 1], b0[k - i - 1], x1, a1[i], b1[k - i], a1[i + 1], b1[k - i - 1]);
      else
        mad64x4(x0, a0[i], b0[k - i], a0[i + 1], b0[k - i - 1], x1, a1[i], b1[k - i], a1[i + 1], b1[k - i - 1]);
      first = false;
      continue;
    }
#endif
    if (first)
      mad64x2_z<false, true>(x0, a0[i], b0[k - i], x1, a1[i], b1[k - i]);
    else
      mad64x2(x0, a0[i], b0[k - i], x1, a1[i], b1[k - i]);
    first = false;
#ifdef ECG_RR_NO_X4
    if (i + 1 <= hi) mad64x2(x0, a0[i + 1], b0[k - i - 1], x1, a1[i + 1], b1[k - i - 1]);
#endif
  }
}
template <class Q>
ECG_DEV void col2p(int k, int lo, int hi, uint64_t& x0, const uint32_t* m0, uint64_t& x1, const uint32_t* m1) {
#if !defined(ECG_RR_NO_X4) && !defined(ECG_RR_X4_ONLY)
  for (; lo + 3 <= hi; lo += 4) {
    const uint32_t t0[4] = {m0[lo], m0[lo + 1], m0[lo + 2], m0[lo + 3]};
    const uint32_t t1[4] = {m1[lo], m1[lo + 1], m1[lo + 2], m1[lo + 3]};
    const uint32_t u[4] = {Q::P[k - lo], Q::P[k - lo - 1], Q::P[k - lo - 2], Q::P[k - lo - 3]};
    mad64x8s(x0, t0, x1, t1, u);
  }
#endif
#pragma unroll
  for (int i = lo; i <= hi; i += 2) {
#ifndef ECG_RR_NO_X4
    if (i + 1 <= hi) {
      mad64x4s(x0, m0[i], m0[i + 1], x1, m1[i], m1[i + 1], Q::P[k - i], Q::P[k - i - 1]);
      continue;
    }
#endif
    mad64x2s(x0, m0[i], x1, m1[i], Q::P[k - i]);
#ifdef ECG_RR_NO_X4
    if (i + 1 <= hi) mad64x2s(x0, m0[i + 1], x1, m1[i + 1], Q::P[k - i - 1]);
#endif
  }
}

// r0 = a0 b0 / R', r1 = a1 b1 / R'
template <class Q>
ECG_DEV void rr_mul2(const FpR<Q>& a0, const FpR<Q>& b0, const FpR<Q>& a1, const FpR<Q>& b1, FpR<Q>& r0,
                     FpR<Q>& r1) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m0[NL], m1[NL];
  uint64_t x0, x1;
  if constexpr (rr_ceil_carry<Q>())
    mad64x2_m1(x0, a0.v[0], b0.v[0], x1, a1.v[0], b1.v[0]);  // column 0 starts both chains at -1
  else
    mad64x2_z<true, true>(x0, a0.v[0], b0.v[0], x1, a1.v[0], b1.v[0]);  // column 0 starts both chains
#pragma unroll
  for (int k = 0; k < NL; k++) {
    if (k > 0) col2(k, 0, k, x0, a0.v, b0.v, x1, a1.v, b1.v);
    uint64_t h0 = 0, h1 = 0;
    if (rr_col_split<Q>(k)) {
      rr_split<Q>(x0, h0);
      rr_split<Q>(x1, h1);
    }
    col2p<Q>(k, 0, k - 1, x0, m0, x1, m1);
    if constexpr (rr_ceil_carry<Q>()) {
      rr_ceil_step<Q>(x0, m0[k], k == NL - 1);
      rr_ceil_step<Q>(x1, m1[k], k == NL - 1);
    } else {
      m0[k] = ((uint32_t)x0 * Q::INV) & MASK;
      m1[k] = ((uint32_t)x1 * Q::INV) & MASK;
      mad64x2s(x0, m0[k], x1, m1[k], Q::P[0]);
      x0 >>= B;
      x1 >>= B;
      if (rr_col_split<Q>(k)) {
        rr_join<Q>(x0, h0);
        rr_join<Q>(x1, h1);
      }
    }
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    col2(k, k - NL + 1, NL - 1, x0, a0.v, b0.v, x1, a1.v, b1.v);
    uint64_t h0 = 0, h1 = 0;
    if (rr_col_split<Q>(k)) {
      rr_split<Q>(x0, h0);
      rr_split<Q>(x1, h1);
    }
    col2p<Q>(k, k - NL + 1, NL - 1, x0, m0, x1, m1);
    r0.v[k - NL] = (uint32_t)x0 & MASK;
    r1.v[k - NL] = (uint32_t)x1 & MASK;
    x0 >>= B;
    x1 >>= B;
    if (rr_col_split<Q>(k)) {
      rr_join<Q>(x0, h0);
      rr_join<Q>(x1, h1);
    }
  }
  r0.v[NL - 1] = (uint32_t)x0;
  r1.v[NL - 1] = (uint32_t)x1;
}

ECG_DEV void mad64x2ss(uint64_t& acc0, uint32_t a0, uint32_t b0_uniform, uint64_t& acc1, uint32_t a1,
                       uint32_t b1_uniform) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_mad_u64_u32 %1, %3, %6, %7, %1"
      : "+v"(acc0), "+v"(acc1), "=&s"(c0), "=&s"(c1)
      : "v"(a0), "s"(b0_uniform), "v"(a1), "s"(b1_uniform));
}

// (a b + c d) / R': one Montgomery reduction for a sum of two products (all
// four operands QN; a column holds 3 NL products < 3 * 14 * 2^58 < 2^64).
// Two accumulators per column (a b | c d, the m p terms split between them)
// merged before the digit.
template <class Q>
ECG_DEV FpR<Q> rr_mul_sum2(const FpR<Q>& a, const FpR<Q>& b, const FpR<Q>& c, const FpR<Q>& d) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m[NL];
  FpR<Q> r;
  uint64_t x0, x1;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    const int i0 = k < NL ? 0 : k - NL + 1;
    const int i1 = k < NL ? k : NL - 1;
    if (k == 0)  // both chains start at zero
      mad64x2_z<true, true>(x0, a.v[0], b.v[0], x1, c.v[0], d.v[0]);
    else  // chain 1 restarts at zero in every column
      col2<true>(k, i0, i1, x0, a.v, b.v, x1, c.v, d.v);
    // BITS = 30: three product sets per column -- split both chains after
    // a b | c d and restart chain 1 for its half of the m p products
    const bool sp = rr_col_split<Q>(k, 2);
    uint64_t h = 0;
    if (sp) {
      uint64_t h1;
      rr_split<Q>(x0, h);
      rr_split<Q>(x1, h1);
      h += h1;
      x0 += x1;
      x1 = 0;
    }
    const int j1 = k < NL ? k - 1 : NL - 1;  // m[j] p[k-j], j in [i0, j1]
    int j = i0;
#pragma unroll
    for (; j + 1 <= j1; j += 2) mad64x2ss(x0, m[j], Q::P[k - j], x1, m[j + 1], Q::P[k - j - 1]);
    if (j == j1) mad64s(x0, m[j], Q::P[k - j]);
    x0 += x1;
    if (k < NL) {
      m[k] = ((uint32_t)x0 * Q::INV) & MASK;
      mad64s(x0, m[k], Q::P[0]);
    } else {
      r.v[k - NL] = (uint32_t)x0 & MASK;
    }
    x0 >>= B;
    if (sp) rr_join<Q>(x0, h);
  }
  r.v[NL - 1] = (uint32_t)x0;
  return r;
}

// r0 = a0^2 / R', r1 = a1^2 / R'
template <class Q>
ECG_DEV void rr_sqr2(const FpR<Q>& a0, const FpR<Q>& a1, FpR<Q>& r0, FpR<Q>& r1) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m0[NL], m1[NL], d0[NL], d1[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    d0[i] = a0.v[i] + a0.v[i];
    d1[i] = a1.v[i] + a1.v[i];
  }
  uint64_t x0, x1;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    const int i0 = k < NL ? 0 : k - NL + 1;
    col2(k, i0, (k & 1) ? k / 2 : k / 2 - 1, x0, d0, a0.v, x1, d1, a1.v);  // 2 i < k
    if (k == 0)  // column 0 (no off-diagonal term) starts both chains
      mad64x2_z<true, true>(x0, a0.v[0], a0.v[0], x1, a1.v[0], a1.v[0]);
    else if ((k & 1) == 0)
      mad64x2(x0, a0.v[k >> 1], a0.v[k >> 1], x1, a1.v[k >> 1], a1.v[k >> 1]);
    uint64_t h0 = 0, h1 = 0;
    if (rr_col_split<Q>(k)) {
      rr_split<Q>(x0, h0);
      rr_split<Q>(x1, h1);
    }
    if (k < NL) {
      col2p<Q>(k, 0, k - 1, x0, m0, x1, m1);
      m0[k] = ((uint32_t)x0 * Q::INV) & MASK;
      m1[k] = ((uint32_t)x1 * Q::INV) & MASK;
      mad64x2s(x0, m0[k], x1, m1[k], Q::P[0]);
    } else {
      col2p<Q>(k, k - NL + 1, NL - 1, x0, m0, x1, m1);
      r0.v[k - NL] = (uint32_t)x0 & MASK;
      r1.v[k - NL] = (uint32_t)x1 & MASK;
    }
    x0 >>= B;
    x1 >>= B;
    if (rr_col_split<Q>(k)) {
      rr_join<Q>(x0, h0);
      rr_join<Q>(x1, h1);
    }
  }
  r0.v[NL - 1] = (uint32_t)x0;
  r1.v[NL - 1] = (uint32_t)x1;
}

// Squaring: off-diagonal products once, against a doubled operand (2 a_i <
// 2^(BITS+1) + 16 keeps every product < 2^59): ~NL^2/2 fewer products.
template <class Q>
ECG_DEV FpR<Q> rr_sqr(const FpR<Q>& a) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t m[NL], a2[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) a2[i] = a.v[i] + a.v[i];
  FpR<Q> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    const int i0 = k < NL ? 0 : k - NL + 1;
#pragma unroll
    for (int i = i0; 2 * i < k; i++) mad64(acc, a2[i], a.v[k - i]);
    if ((k & 1) == 0) mad64(acc, a.v[k >> 1], a.v[k >> 1]);
    uint64_t h = 0;
    if (rr_col_split<Q>(k)) rr_split<Q>(acc, h);
    if (k < NL) {
#pragma unroll
      for (int i = 0; i < k; i++) mad64s(acc, m[i], Q::P[k - i]);
      m[k] = ((uint32_t)acc * Q::INV) & MASK;
      mad64s(acc, m[k], Q::P[0]);
    } else {
#pragma unroll
      for (int i = k - NL + 1; i < NL; i++) mad64s(acc, m[i], Q::P[k - i]);
      r.v[k - NL] = (uint32_t)acc & MASK;
    }
    acc >>= B;
    if (rr_col_split<Q>(k)) rr_join<Q>(acc, h);
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// One parallel carry step: limb i keeps its low BITS bits plus the carry of
// limb i-1 (s[i] < 2^32 on entry -> QN on exit); the top limb keeps all bits.
template <class Q>
ECG_DEV FpR<Q> rr_carry(const uint32_t* s) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  FpR<Q> r;
  r.v[0] = s[0] & MASK;
#pragma unroll
  for (int i = 1; i < NL - 1; i++) r.v[i] = (s[i] & MASK) + (s[i - 1] >> B);
  r.v[NL - 1] = s[NL - 1] + (s[NL - 2] >> B);
  return r;
}

template <class Q>
ECG_DEV FpR<Q> rr_add(const FpR<Q>& a, const FpR<Q>& b) {
  uint32_t s[Q::NL];
#pragma unroll
  for (int i = 0; i < Q::NL; i++) s[i] = a.v[i] + b.v[i];
  return rr_carry<Q>(s);
}

template <int K>
constexpr int kp_index() {
  static_assert(K >= 2 && (K & (K - 1)) == 0 && K <= 256, "k must be a power of two in [2, 256]");
  return K == 2 ? 0 : K == 4 ? 1 : K == 8 ? 2 : K == 16 ? 3 : K == 32 ? 4 : K == 64 ? 5 : K == 128 ? 6 : 7;
}

// a - b + K p  (requires value(b) <= K p / 2)
template <int K, class Q>
ECG_DEV FpR<Q> rr_sub(const FpR<Q>& a, const FpR<Q>& b) {
  constexpr int j = kp_index<K>();
  static_assert((Q::KP_OK >> j) & 1, "K p not representable for this field (tools/gen_params_rr.py)");
  uint32_t s[Q::NL];
#pragma unroll
  for (int i = 0; i < Q::NL; i++) s[i] = a.v[i] + Q::KP[j][i] - b.v[i];
  return rr_carry<Q>(s);
}

// K p - a  (requires value(a) <= K p / 2)
template <int K, class Q>
ECG_DEV FpR<Q> rr_neg(const FpR<Q>& a) {
  constexpr int j = kp_index<K>();
  static_assert((Q::KP_OK >> j) & 1, "K p not representable for this field (tools/gen_params_rr.py)");
  uint32_t s[Q::NL];
#pragma unroll
  for (int i = 0; i < Q::NL; i++) s[i] = Q::KP[j][i] - a.v[i];
  return rr_carry<Q>(s);
}

// a + K p - b - c - d  (deep-borrowed K p; requires b + c + d <= K p / 2):
// three subtractions, one carry step
template <int K, class Q>
ECG_DEV FpR<Q> rr_sub3(const FpR<Q>& a, const FpR<Q>& b, const FpR<Q>& c, const FpR<Q>& d) {
  constexpr int j = kp_index<K>();
  if constexpr (Q::BITS > 29) {  // no deep borrow in 32-bit limbs: sum the subtrahends first
    return rr_sub<K>(a, rr_add(b, rr_add(c, d)));
  }
  static_assert(Q::BITS > 29 || ((Q::KPD_OK >> j) & 1), "K p (deep borrow) not representable for this field");
  uint32_t s[Q::NL];
#pragma unroll
  for (int i = 0; i < Q::NL; i++) s[i] = a.v[i] + Q::KPD[j][i] - b.v[i] - c.v[i] - d.v[i];
  return rr_carry<Q>(s);
}

// a + K p - b - c
template <int K, class Q>
ECG_DEV FpR<Q> rr_sub2(const FpR<Q>& a, const FpR<Q>& b, const FpR<Q>& c) {
  constexpr int j = kp_index<K>();
  if constexpr (Q::BITS > 29) {
    return rr_sub<K>(a, rr_add(b, c));
  }
  static_assert(Q::BITS > 29 || ((Q::KPD_OK >> j) & 1), "K p (deep borrow) not representable for this field");
  uint32_t s[Q::NL];
#pragma unroll
  for (int i = 0; i < Q::NL; i++) s[i] = a.v[i] + Q::KPD[j][i] - b.v[i] - c.v[i];
  return rr_carry<Q>(s);
}

// K p - a WITHOUT the carry step ("wide": limbs < 2^(BITS+1) + 2^BITS).  Only
// for an operand of rr_mul / rr_mul2 whose partner is a product output: the
// column then stays below 14 * 2^59.6 + 14 * 2^58 < 2^64.
template <int K, class Q>
ECG_DEV FpR<Q> rr_neg_wide(const FpR<Q>& a) {
  constexpr int j = kp_index<K>();
  static_assert((Q::KP_OK >> j) & 1, "K p not representable for this field (tools/gen_params_rr.py)");
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = Q::KP[j][i] - a.v[i];
  return r;
}

// exact all-zero limbs (the identity marker; never a product output of a
// non-zero value)
template <class Q>
ECG_DEV bool fis_zero(const FpR<Q>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) o |= a.v[i];
  return o == 0;
}

// v == 0 (mod p) for a product output (exact limbs, value < 2p)
template <class Q>
ECG_DEV bool rr_is_zero_prod(const FpR<Q>& a) {
  uint32_t o = 0, q = 0;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) {
    o |= a.v[i];
    q |= a.v[i] ^ Q::P[i];
  }
  return o == 0 || q == 0;
}

// cheap necessary condition for rr_is_zero_prod (low limb only): lets the
// rare exceptional paths sit behind a wave-uniform branch
template <class Q>
ECG_DEV bool rr_maybe_zero_prod(const FpR<Q>& a) {
  return a.v[0] == 0 || a.v[0] == Q::P[0];
}

// ---------------------------------------------------------------------------
// radix change: 32-bit words <-> BITS-bit limbs (exact integers)
// ---------------------------------------------------------------------------
template <class Q, int L>
ECG_DEV void rr_unpack(const uint32_t* w, uint32_t* limb) {
  constexpr int B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) {
    const int bit = B * i, j = bit >> 5, s = bit & 31;
    uint32_t v = j < L ? w[j] >> s : 0u;
    if (s != 0 && 32 - s < B && j + 1 < L) v |= w[j + 1] << (32 - s);
    limb[i] = v & MASK;
  }
}

template <class Q, int L>
ECG_DEV void rr_pack(const uint32_t* limb, uint32_t* w) {
  constexpr int B = Q::BITS;
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int bit = 32 * j, i = bit / B, s = bit % B;
    uint32_t v = i < Q::NL ? limb[i] >> s : 0u;
    if (B - s < 32 && i + 1 < Q::NL) v |= limb[i + 1] << (B - s);
    if (2 * B - s < 32 && i + 2 < Q::NL) v |= limb[i + 2] << (2 * B - s);
    w[j] = v;
  }
}

// ark-ff Montgomery (x R, 32-bit limbs, < p) -> x R' (product output form)
template <class Q>
ECG_DEV FpR<Q> rr_from_std(const Fp<typename Q::Base>& a) {
  FpR<Q> x, c;
  rr_unpack<Q, Fp<typename Q::Base>::L>(a.v, x.v);
#pragma unroll
  for (int i = 0; i < Q::NL; i++) c.v[i] = Q::TO_RR[i];
  return rr_mul(x, c);
}

// x R' (any lazy value <= 64 p) -> canonical ark-ff Montgomery x R (< p)
template <class Q>
ECG_DEV Fp<typename Q::Base> rr_to_std(const FpR<Q>& a) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  FpR<Q> c;
#pragma unroll
  for (int i = 0; i < NL; i++) c.v[i] = Q::FROM_RR[i];
  FpR<Q> y = rr_mul(a, c);  // x R, exact limbs, value < 2p
  uint32_t t[NL];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {  // t = y - p, sequential borrow
    const int32_t d = (int32_t)y.v[i] - (int32_t)Q::P[i] + br;
    t[i] = (uint32_t)d & MASK;
    br = d >> B;  // 0 or -1
  }
  const bool ge = br == 0;
#pragma unroll
  for (int i = 0; i < NL; i++) y.v[i] = ge ? t[i] : y.v[i];
  Fp<typename Q::Base> r;
  rr_pack<Q, Fp<typename Q::Base>::L>(y.v, r.v);
  return r;
}

// ---------------------------------------------------------------------------
// carry-free sums / differences and cheap value reduction (the NTT's
// butterflies, ntt.hip; bounds in the NTT section of DESIGN.md)
// ---------------------------------------------------------------------------
// a + b, limb by limb (no carry step)
template <class Q>
ECG_DEV FpR<Q> rr_add_nc(const FpR<Q>& a, const FpR<Q>& b) {
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// a + K p - b, limb by limb (no carry step): limb-wise non-negative when every
// limb of b is <= 2^(BITS+1) - 2 and value(b) <= K p / 2
template <int K, class Q>
ECG_DEV FpR<Q> rr_sub_nc(const FpR<Q>& a, const FpR<Q>& b) {
  constexpr int j = kp_index<K>();
  static_assert((Q::KP_OK >> j) & 1, "K p not representable for this field (tools/gen_params_rr.py)");
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = a.v[i] + Q::KP[j][i] - b.v[i];
  return r;
}

// Exact limbs (< 2^BITS below the top limb), same value: sequential carry.
template <class Q>
ECG_DEV FpR<Q> rr_carry_seq(const FpR<Q>& a) {
  constexpr int B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  FpR<Q> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < Q::NL - 1; i++) {
    const uint64_t t = (uint64_t)a.v[i] + c;
    r.v[i] = (uint32_t)t & MASK;
    c = (uint32_t)(t >> B);
  }
  r.v[Q::NL - 1] = a.v[Q::NL - 1] + c;
  return r;
}

// v - q p with q = floor(v_top * floor(2^32 / (P_top + 1)) / 2^32), never
// above floor(v / p): for limbs < 2^31.4 and value < 64 p the result has
// exact limbs and value < p (1 + v_top / 2^32) + 2^(BITS (NL-1) + 6) < 1.1 p
// -- a product-free "mod p, almost".
template <class Q>
ECG_DEV FpR<Q> rr_reduce_q(const FpR<Q>& a) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  constexpr uint32_t MAGIC = (uint32_t)((1ull << 32) / ((uint64_t)Q::P[NL - 1] + 1));
  const uint32_t q = __umulhi(a.v[NL - 1], MAGIC);
  FpR<Q> r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    const int64_t t = (int64_t)a.v[i] + c - (int64_t)((uint64_t)q * Q::P[i]);
    r.v[i] = (uint32_t)t & MASK;
    c = t >> B;  // arithmetic
  }
  r.v[NL - 1] = (uint32_t)((int64_t)a.v[NL - 1] + c - (int64_t)((uint64_t)q * Q::P[NL - 1]));
  return r;
}

// Canonical value (< p) of an exact-limb value < 2p: one conditional
// subtraction with a sequential borrow.
template <class Q>
ECG_DEV FpR<Q> rr_canon_lt2p(const FpR<Q>& a) {
  constexpr int NL = Q::NL, B = Q::BITS;
  constexpr uint32_t MASK = (1u << B) - 1;
  uint32_t t[NL];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int32_t d = (int32_t)a.v[i] - (int32_t)Q::P[i] + br;
    t[i] = i + 1 < NL ? (uint32_t)d & MASK : (uint32_t)d;
    br = d >> B;  // 0 or -1 (top limb: sign of the difference)
  }
  const bool ge = br == 0;
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = ge ? t[i] : a.v[i];
  return r;
}

// ---------------------------------------------------------------------------
// memory: NL words, moved as 16-B vectors where NL allows
// ---------------------------------------------------------------------------
template <class Q>
ECG_DEV FpR<Q> load(const FpR<Q>* p) {
  FpR<Q> r;
  if constexpr (Q::NL % 2 == 0) {
    const uint2* s = reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < Q::NL / 2; i++) {
      const uint2 t = s[i];
      r.v[2 * i] = t.x;
      r.v[2 * i + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < Q::NL; i++) r.v[i] = p->v[i];
  }
  return r;
}

template <class Q>
ECG_DEV void store(FpR<Q>* p, const FpR<Q>& a) {
  if constexpr (Q::NL % 2 == 0) {
    uint2* d = reinterpret_cast<uint2*>(p);
#pragma unroll
    for (int i = 0; i < Q::NL / 2; i++) d[i] = make_uint2(a.v[2 * i], a.v[2 * i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < Q::NL; i++) p->v[i] = a.v[i];
  }
}

}  // namespace ecg
