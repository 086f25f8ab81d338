// XYZZ point arithmetic over the reduced-radix field (fieldrr.hpp) for the
// MSM bucket pipeline: the same formulas as curve.hpp (madd-2008-s,
// add-2008-s, dbl-2008-s-1 / mdbl-2008-s-1; ec.cl:17-130's role), with every
// subtraction's multiple of p chosen from a value bound, so no value ever
// needs a conditional reduction.  Bounds, in units of p (product outputs
// M < 1.01 p given the >= 2^25 slack):
//   stored points  X <= 17.01, Y <= 4.01, ZZ, ZZZ <= M;  bases x, y <= M,
//                  a negated base y is 4p - y (<= 4p, "wide" limbs)
//   madd:  P = U2 - X1 + 64p <= 65, R = S2 - Y1 + 16p <= 17,
//          X3 = R^2 - PPP - 2Q + 16p <= 17.01, D = Q - X3 + 64p <= 65,
//          Y3 = (R D + Y1 (4p - PPP)) / R'  (one reduction for both
//          products) <= M
//   add:   P, R <= 5.01 (+4p), the rest as madd
//   dbl:   U = 2Y <= 8.02, M = 3X^2 <= 3.03, X3, Y3 as madd
// Largest product of operand bounds: 65 x 65 = 4225 << 2^24.
//
// Tight-slack layouts (rr_tight: R'/p < 2^16 -- BN254's 9 x 29-bit G1 form,
// R'/p ~ 167.8, chosen over 10 x 28 bits for 162 instead of 200 mads per
// product) cannot afford those operands: a product output is
// < a b / R' + p, so operands must multiply to well under 168 p^2.  There X3
// is brought back to ~p by rr_reduce_q (a product-free "mod p, almost") and
// every subtraction uses 4p, which bounds everything by:
//   stored points  X <= 1.02 (reduced), Y <= 1.25, ZZ, ZZZ <= M;  M < 1.25 p
//                  (largest product below 35 p^2); bases x, y <= M, a
//                  negated base y is 4p - y (<= 4p, wide limbs)
//   madd:  P = U2 - X1 + 4p <= 5.3, R = S2 - Y1 + 4p <= 5.3, RR, PP <= 1.17,
//          X3 = reduce_q(RR - PPP - 2Q + 16p) <= 1.02, D = Q - X3 + 4p <= 5.3,
//          Y3 = (R D + Y1 (4p - PPP)) / R' <= 1.21
//   add:   the same with U1 for X1 and S1 for Y1
//   dbl:   U = 2Y <= 8 (a wide base y in the doubling branch), V <= 1.39,
//          M = 3X^2 <= 3.6, X3 reduced, Y3 = (M D + Y (4p - W)) / R' <= 1.21
//   a stored Y never comes from a wide value unreduced (the first base of a
//   bucket, a negation) -- rr_reduce_q takes it to <= 1.02.
// Exceptional cases (P = 0 mod p: doubling or inverse) are detected on PP =
// P^2, a product output, whose low limb screens them behind a branch that
// waves almost never take.  The identity is the all-zero ZZ marker.
#pragma once
#include "curve.hpp"
#include "fieldrr.hpp"

namespace ecg {

template <class Q>
constexpr bool rr_tight() {
  return Q::SLACK_LOG2 < 16;
}

template <class Q>
ECG_DEV bool xyzz_is_zero_rr(const XYZZ<FpR<Q>>& p) {
  return fis_zero(p.ZZ);
}

// dbl-2008-s-1 core on (X, Y) with the new ZZ, ZZZ factors V = U^2, W = U V
template <class Q>
ECG_DEV void rr_dbl_core(const FpR<Q>& X, const FpR<Q>& Y, XYZZ<FpR<Q>>& r, FpR<Q>& V, FpR<Q>& W) {
  using F = FpR<Q>;
  const F U = rr_add(Y, Y);
  F S, X2;
  rr_sqr2(U, X, V, X2);  // the two independent squarings as one interleaved pair
  rr_mul2(U, V, X, V, W, S);
  const F Mm = rr_add(rr_add(X2, X2), X2);
  if constexpr (rr_tight<Q>()) {
    r.X = rr_reduce_q(rr_sub2<16>(rr_sqr(Mm), S, S));
    r.Y = rr_mul_sum2(Mm, rr_sub<4>(S, r.X), Y, rr_neg<4>(W));
  } else {
    r.X = rr_sub2<16>(rr_sqr(Mm), S, S);
    r.Y = rr_mul_sum2(Mm, rr_sub<64>(S, r.X), Y, rr_neg<4>(W));
  }
}

// mdbl-2008-s-1: 2 (x, y)
template <class Q>
ECG_DEV XYZZ<FpR<Q>> rr_dbl_affine(const Affine<FpR<Q>>& a) {
  XYZZ<FpR<Q>> r;
  rr_dbl_core(a.x, a.y, r, r.ZZ, r.ZZZ);
  return r;
}

// dbl-2008-s-1: 2 P
template <class Q>
ECG_DEV XYZZ<FpR<Q>> rr_dbl(const XYZZ<FpR<Q>>& p) {
  using F = FpR<Q>;
  if (xyzz_is_zero_rr(p)) return p;
  XYZZ<F> r;
  F V, W;
  rr_dbl_core(p.X, p.Y, r, V, W);
  rr_mul2(V, p.ZZ, W, p.ZZZ, r.ZZ, r.ZZZ);
  return r;
}

// r = c ? s : r, limb by limb.  Results are merged this way (single exit, no
// whole-struct assignment under a condition): a struct copy from a selected
// source becomes a copy through a selected pointer, which pins both points
// in scratch memory (measured: ~300 GB of scratch traffic per 2^26 MSM).
template <class Q>
ECG_DEV void rr_sel(FpR<Q>& r, bool c, const FpR<Q>& s) {
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = c ? s.v[i] : r.v[i];
}
template <class Q>
ECG_DEV void rr_sel(XYZZ<FpR<Q>>& r, bool c, const XYZZ<FpR<Q>>& s) {
  rr_sel(r.X, c, s.X);
  rr_sel(r.Y, c, s.Y);
  rr_sel(r.ZZ, c, s.ZZ);
  rr_sel(r.ZZZ, c, s.ZZZ);
}

// madd-2008-s: P + (x2, y2); `a` must not be the identity (a.y may be wide).
// Products run as independent pairs (rr_mul2 / rr_sqr2) plus one product sum.
template <class Q>
ECG_DEV XYZZ<FpR<Q>> rr_add_affine(const XYZZ<FpR<Q>>& p, const Affine<FpR<Q>>& a) {
  using F = FpR<Q>;
  XYZZ<F> r;
  // a.y (possibly wide) is carried only where it becomes a stored coordinate
  // (stored points are QN); the common path feeds it straight into a product
  constexpr bool tight = rr_tight<Q>();
  if (xyzz_is_zero_rr(p)) {
    r.X = a.x;
    r.Y = rr_carry<Q>(a.y.v);
    if constexpr (tight) r.Y = rr_reduce_q(r.Y);
    r.ZZ = F::one();
    r.ZZZ = F::one();
  } else {
    F U2, S2, PP, RR, PPP, Qv;
    rr_mul2(a.x, p.ZZ, a.y, p.ZZZ, U2, S2);
    F P, R;
    if constexpr (tight) {
      P = rr_sub<4>(U2, p.X);
      R = rr_sub<4>(S2, p.Y);
    } else {
      P = rr_sub<64>(U2, p.X);
      R = rr_sub<16>(S2, p.Y);
    }
    rr_sqr2(P, R, PP, RR);
    rr_mul2(P, PP, p.X, PP, PPP, Qv);
    rr_mul2(p.ZZ, PP, p.ZZZ, PPP, r.ZZ, r.ZZZ);
    if constexpr (tight) {
      r.X = rr_reduce_q(rr_sub3<16>(RR, PPP, Qv, Qv));
      r.Y = rr_mul_sum2(R, rr_sub<4>(Qv, r.X), p.Y, rr_neg<4>(PPP));
    } else {
      r.X = rr_sub3<16>(RR, PPP, Qv, Qv);
      r.Y = rr_mul_sum2(R, rr_sub<64>(Qv, r.X), p.Y, rr_neg<4>(PPP));
    }
    if (rr_maybe_zero_prod(PP)) {  // rare: P = Q or P = -Q
      const bool inf = rr_is_zero_prod(PP);
      const bool dbl = inf && rr_is_zero_prod(RR);
      XYZZ<F> d = xyzz_zero<F>();
      if (dbl) {
        Affine<F> b;
        b.x = a.x;
        b.y = rr_carry<Q>(a.y.v);
        d = rr_dbl_affine(b);
      }
      rr_sel(r, inf, d);
    }
  }
  return r;
}

// add-2008-s: P + Q
template <class Q>
ECG_DEV XYZZ<FpR<Q>> rr_add_xyzz(const XYZZ<FpR<Q>>& p, const XYZZ<FpR<Q>>& q) {
  using F = FpR<Q>;
  const bool pz = xyzz_is_zero_rr(p), qz = xyzz_is_zero_rr(q);
  XYZZ<F> r;
  if (pz || qz) {  // single exit, limb selects (see rr_sel)
    r = q;
    rr_sel(r, qz, p);
  } else {
    F U1, U2, S1, S2, PP, RR, PPP, Qv, ZZ12, ZZZ12;
    rr_mul2(p.X, q.ZZ, q.X, p.ZZ, U1, U2);
    rr_mul2(p.Y, q.ZZZ, q.Y, p.ZZZ, S1, S2);
    const F P = rr_sub<4>(U2, U1);
    const F R = rr_sub<4>(S2, S1);
    rr_sqr2(P, R, PP, RR);
    rr_mul2(P, PP, U1, PP, PPP, Qv);
    rr_mul2(p.ZZ, q.ZZ, p.ZZZ, q.ZZZ, ZZ12, ZZZ12);
    rr_mul2(ZZ12, PP, ZZZ12, PPP, r.ZZ, r.ZZZ);
    if constexpr (rr_tight<Q>()) {
      r.X = rr_reduce_q(rr_sub3<16>(RR, PPP, Qv, Qv));
      r.Y = rr_mul_sum2(R, rr_sub<4>(Qv, r.X), S1, rr_neg<4>(PPP));
    } else {
      r.X = rr_sub3<16>(RR, PPP, Qv, Qv);
      r.Y = rr_mul_sum2(R, rr_sub<64>(Qv, r.X), S1, rr_neg<4>(PPP));
    }
    if (rr_maybe_zero_prod(PP)) {
      const bool inf = rr_is_zero_prod(PP);
      const bool dbl = inf && rr_is_zero_prod(RR);
      XYZZ<F> d = xyzz_zero<F>();
      if (dbl) d = rr_dbl(p);
      rr_sel(r, inf, d);
    }
  }
  return r;
}

// ---------------------------------------------------------------------------
// Lane-pair forms for latency-bound chains.  A wave issues at most one VALU
// instruction every ~2 quad-cycles when it is alone on its SIMD
// (profiles/r04/mad_latency.txt: ~4 ns per v_mad_u64_u32 for one wave, with 1
// to 8 independent chains alike), so a chain of point operations at under one
// wave per SIMD runs at about half the issue rate whatever its ILP.  Fewer
// instructions per wave per operation is what shortens it: two lanes (the
// pair lane ^ M, M = 1 or 2) hold the same operands and each computes half of
// every level's products, exchanging results through DPP quad permutes.  The
// values are those of rr_dbl / rr_add_xyzz (same formulas, same bounds), only
// distributed; both lanes return the whole result.  Both lanes of a pair must
// run the call together (pair-uniform control flow).
// ---------------------------------------------------------------------------
template <int M>
ECG_DEV uint32_t lane_swap_u32(uint32_t v) {
  static_assert(M == 1 || M == 2, "pairs are lanes ^ 1 or lanes ^ 2 of a quad");
  // quad_perm [1,0,3,2] (0xB1) or [2,3,0,1] (0x4E)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, M == 1 ? 0xB1 : 0x4E, 0xF, 0xF, false);
}
template <int M, class Q>
ECG_DEV FpR<Q> rr_lane_swap(const FpR<Q>& a) {
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = lane_swap_u32<M>(a.v[i]);
  return r;
}
template <class Q>
ECG_DEV FpR<Q> rr_pick(bool c, const FpR<Q>& a, const FpR<Q>& b) {  // c ? a : b
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}
template <int M>
ECG_DEV bool pair_hi() {
  return (threadIdx.x & M) != 0;
}

// 2 P (dbl-2008-s-1, as rr_dbl) on a lane pair.  Lane lo / hi:
//   level 1: V = U^2          | X2 = X^2
//   level 2: W = U V, ZZ3 = V ZZ | S = X V, M^2
//   level 3: ZZZ3 = W ZZZ      | Y3 = M (S - X3) + Y (k p - W)
// with three exchanges (V | X2, W | S, then the outputs).
template <int M, class Q>
ECG_DEV XYZZ<FpR<Q>> rr_dbl_x2(const XYZZ<FpR<Q>>& p) {
  using F = FpR<Q>;
  if (xyzz_is_zero_rr(p)) return p;
  const bool h = pair_hi<M>();
  const F U = rr_add(p.Y, p.Y);
  const F L1 = rr_sqr(rr_pick(h, p.X, U));
  const F O1 = rr_lane_swap<M>(L1);
  const F V = rr_pick(h, O1, L1), X2 = rr_pick(h, L1, O1);
  const F Mm = rr_add(rr_add(X2, X2), X2);
  F a0, a1;
  rr_mul2(rr_pick(h, p.X, U), V, rr_pick(h, Mm, V), rr_pick(h, Mm, p.ZZ), a0, a1);
  const F O2 = rr_lane_swap<M>(a0);
  const F W = rr_pick(h, O2, a0), S = rr_pick(h, a0, O2);
  F X3, D;  // meaningful on the hi lane (a1 = M^2 there)
  if constexpr (rr_tight<Q>()) {
    X3 = rr_reduce_q(rr_sub2<16>(a1, S, S));
    D = rr_sub<4>(S, X3);
  } else {
    X3 = rr_sub2<16>(a1, S, S);
    D = rr_sub<64>(S, X3);
  }
  const F z = F::zero();
  const F r = rr_mul_sum2(rr_pick(h, Mm, W), rr_pick(h, D, p.ZZZ), rr_pick(h, p.Y, z), rr_pick(h, rr_neg<4>(W), z));
  const F f = rr_lane_swap<M>(r);                   // lo <- Y3, hi <- ZZZ3
  const F g = rr_lane_swap<M>(rr_pick(h, X3, a1));  // lo <- X3, hi <- ZZ3
  XYZZ<F> o;
  o.X = rr_pick(h, X3, g);
  o.Y = rr_pick(h, r, f);
  o.ZZ = rr_pick(h, g, a1);
  o.ZZZ = rr_pick(h, f, r);
  return o;
}

// P + Q (add-2008-s, as rr_add_xyzz) on a lane pair.  Lane lo / hi:
//   level 1: U1 = X1 ZZ2, S1 = Y1 ZZZ2   | U2 = X2 ZZ1, S2 = Y2 ZZZ1
//   level 2: PP = P^2, RR = R^2          | ZZ12, ZZZ12
//   level 3: PPP = P PP, Q = U1 PP       | ZZ3 = ZZ12 PP
//   level 4: Y3 = R (Q - X3) + S1 (k p - PPP) | ZZZ3 = ZZZ12 PPP
template <int M, class Q>
ECG_DEV XYZZ<FpR<Q>> rr_add_x2(const XYZZ<FpR<Q>>& p, const XYZZ<FpR<Q>>& q) {
  using F = FpR<Q>;
  const bool pz = xyzz_is_zero_rr(p), qz = xyzz_is_zero_rr(q);
  XYZZ<F> o;
  if (pz || qz) {
    o = q;
    rr_sel(o, qz, p);
    return o;
  }
  const bool h = pair_hi<M>();
  F a0, a1;
  rr_mul2(rr_pick(h, q.X, p.X), rr_pick(h, p.ZZ, q.ZZ), rr_pick(h, q.Y, p.Y), rr_pick(h, p.ZZZ, q.ZZZ), a0, a1);
  const F e0 = rr_lane_swap<M>(a0), e1 = rr_lane_swap<M>(a1);
  const F U1 = rr_pick(h, e0, a0), U2 = rr_pick(h, a0, e0);
  const F S1 = rr_pick(h, e1, a1), S2 = rr_pick(h, a1, e1);
  const F P = rr_sub<4>(U2, U1);
  const F R = rr_sub<4>(S2, S1);
  F b0, b1;  // lo: PP, RR | hi: ZZ12, ZZZ12
  rr_mul2(rr_pick(h, p.ZZ, P), rr_pick(h, q.ZZ, P), rr_pick(h, p.ZZZ, R), rr_pick(h, q.ZZZ, R), b0, b1);
  const F e2 = rr_lane_swap<M>(b0);
  const F PP = rr_pick(h, e2, b0), ZZ12 = rr_pick(h, b0, e2);
  F c0, c1;  // lo: PPP, Q | hi: ZZ3 (twice)
  rr_mul2(rr_pick(h, ZZ12, P), PP, rr_pick(h, ZZ12, U1), PP, c0, c1);
  const F e3 = rr_lane_swap<M>(c0);
  const F PPP = rr_pick(h, e3, c0), ZZ3 = rr_pick(h, c0, e3);
  F X3, D;  // meaningful on the lo lane (b1 = RR, c1 = Q there)
  if constexpr (rr_tight<Q>()) {
    X3 = rr_reduce_q(rr_sub3<16>(b1, PPP, c1, c1));
    D = rr_sub<4>(c1, X3);
  } else {
    X3 = rr_sub3<16>(b1, PPP, c1, c1);
    D = rr_sub<64>(c1, X3);
  }
  const F z = F::zero();
  const F r = rr_mul_sum2(rr_pick(h, b1, R), rr_pick(h, PPP, D), rr_pick(h, z, S1), rr_pick(h, z, rr_neg<4>(PPP)));
  const F f = rr_lane_swap<M>(r);   // lo <- ZZZ3, hi <- Y3
  const F g = rr_lane_swap<M>(X3);  // hi <- X3
  o.X = rr_pick(h, g, X3);
  o.Y = rr_pick(h, f, r);
  o.ZZ = ZZ3;
  o.ZZZ = rr_pick(h, r, f);
  if (rr_maybe_zero_prod(PP)) {  // rare, pair-uniform (both lanes hold PP): P = Q or P = -Q
    const F RRv = rr_pick(h, rr_lane_swap<M>(b1), b1);
    const bool inf = rr_is_zero_prod(PP);
    const bool dbl = inf && rr_is_zero_prod(RRv);
    XYZZ<F> d = xyzz_zero<F>();
    if (dbl) d = rr_dbl_x2<M>(p);
    rr_sel(o, inf, d);
  }
  return o;
}

// Quad forms: four lanes (threadIdx & 3) share each operation, one product
// per lane and level, every level's results broadcast to the quad by DPP.
// Per lane a doubling issues 1 squaring + 1 product + 1 product sum (pairs: 1
// + 2 + 1; one lane: 9 products), a full add 3 products + 1 product sum
// (pairs: 6 + 1; one lane: 14).  Same values and bounds as rr_dbl /
// rr_add_xyzz; quad-uniform control flow.
template <int L, class Q>
ECG_DEV FpR<Q> rr_quad_bcast(const FpR<Q>& a) {  // lane L's value on every lane of the quad
  constexpr int ctrl = L | (L << 2) | (L << 4) | (L << 6);  // quad_perm [L, L, L, L]
  FpR<Q> r;
#pragma unroll
  for (int i = 0; i < Q::NL; i++) r.v[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v[i], ctrl, 0xF, 0xF, false);
  return r;
}
template <class Q>
ECG_DEV FpR<Q> rr_pick4(uint32_t q, const FpR<Q>& a0, const FpR<Q>& a1, const FpR<Q>& a2, const FpR<Q>& a3) {
  return rr_pick((q & 2) != 0, rr_pick((q & 1) != 0, a3, a2), rr_pick((q & 1) != 0, a1, a0));
}

// 2 P on a quad.  Lanes 0 / 1 / 2 / 3:
//   level 1: V = U^2 | X2 = X^2 | (V) | (X2)
//   level 2: W = U V | S = X V | ZZ3 = V ZZ | M^2
//   level 3: ZZZ3 = W ZZZ | Y3 = M (S - X3) + Y (k p - W) | (ZZZ3) | (Y3)
template <class Q>
ECG_DEV XYZZ<FpR<Q>> rr_dbl_x4(const XYZZ<FpR<Q>>& p) {
  using F = FpR<Q>;
  if (xyzz_is_zero_rr(p)) return p;
  const uint32_t q = threadIdx.x & 3u;
  const bool odd = (q & 1u) != 0;
  const F U = rr_add(p.Y, p.Y);
  const F L1 = rr_sqr(rr_pick(odd, p.X, U));
  const F V = rr_quad_bcast<0>(L1), X2 = rr_quad_bcast<1>(L1);
  const F Mm = rr_add(rr_add(X2, X2), X2);
  const F a = rr_mul(rr_pick4(q, U, p.X, V, Mm), rr_pick4(q, V, V, p.ZZ, Mm));
  const F W = rr_quad_bcast<0>(a), S = rr_quad_bcast<1>(a), ZZ3 = rr_quad_bcast<2>(a), M2 = rr_quad_bcast<3>(a);
  F X3, D;
  if constexpr (rr_tight<Q>()) {
    X3 = rr_reduce_q(rr_sub2<16>(M2, S, S));
    D = rr_sub<4>(S, X3);
  } else {
    X3 = rr_sub2<16>(M2, S, S);
    D = rr_sub<64>(S, X3);
  }
  const F z = F::zero();
  const F r = rr_mul_sum2(rr_pick(odd, Mm, W), rr_pick(odd, D, p.ZZZ), rr_pick(odd, p.Y, z), rr_pick(odd, rr_neg<4>(W), z));
  XYZZ<F> o;
  o.X = X3;
  o.Y = rr_quad_bcast<1>(r);
  o.ZZ = ZZ3;
  o.ZZZ = rr_quad_bcast<0>(r);
  return o;
}

// P + Q on a quad.  Lanes 0 / 1 / 2 / 3:
//   level 1: U1 = X1 ZZ2 | U2 = X2 ZZ1 | S1 = Y1 ZZZ2 | S2 = Y2 ZZZ1
//   level 2: PP = P^2 | RR = R^2 | ZZ12 | ZZZ12
//   level 3: PPP = P PP | Q = U1 PP | ZZ3 = ZZ12 PP | (ZZ3)
//   level 4: Y3 = R (Q - X3) + S1 (k p - PPP) | ZZZ3 = ZZZ12 PPP | (Y3) | (ZZZ3)
template <class Q>
ECG_DEV XYZZ<FpR<Q>> rr_add_x4(const XYZZ<FpR<Q>>& p, const XYZZ<FpR<Q>>& q2) {
  using F = FpR<Q>;
  const bool pz = xyzz_is_zero_rr(p), qz = xyzz_is_zero_rr(q2);
  XYZZ<F> o;
  if (pz || qz) {
    o = q2;
    rr_sel(o, qz, p);
    return o;
  }
  const uint32_t q = threadIdx.x & 3u;
  const bool odd = (q & 1u) != 0;
  const F a = rr_mul(rr_pick4(q, p.X, q2.X, p.Y, q2.Y), rr_pick4(q, q2.ZZ, p.ZZ, q2.ZZZ, p.ZZZ));
  const F U1 = rr_quad_bcast<0>(a), U2 = rr_quad_bcast<1>(a), S1 = rr_quad_bcast<2>(a), S2 = rr_quad_bcast<3>(a);
  const F P = rr_sub<4>(U2, U1);
  const F R = rr_sub<4>(S2, S1);
  const F b = rr_mul(rr_pick4(q, P, R, p.ZZ, p.ZZZ), rr_pick4(q, P, R, q2.ZZ, q2.ZZZ));
  const F PP = rr_quad_bcast<0>(b), RR = rr_quad_bcast<1>(b), ZZ12 = rr_quad_bcast<2>(b), ZZZ12 = rr_quad_bcast<3>(b);
  const F c = rr_mul(rr_pick4(q, P, U1, ZZ12, ZZ12), PP);
  const F PPP = rr_quad_bcast<0>(c), Qv = rr_quad_bcast<1>(c);
  F X3, D;
  if constexpr (rr_tight<Q>()) {
    X3 = rr_reduce_q(rr_sub3<16>(RR, PPP, Qv, Qv));
    D = rr_sub<4>(Qv, X3);
  } else {
    X3 = rr_sub3<16>(RR, PPP, Qv, Qv);
    D = rr_sub<64>(Qv, X3);
  }
  const F z = F::zero();
  const F r = rr_mul_sum2(rr_pick(odd, ZZZ12, R), rr_pick(odd, PPP, D), rr_pick(odd, z, S1), rr_pick(odd, z, rr_neg<4>(PPP)));
  o.X = X3;
  o.Y = rr_quad_bcast<0>(r);
  o.ZZ = rr_quad_bcast<2>(c);
  o.ZZZ = rr_quad_bcast<1>(r);
  if (rr_maybe_zero_prod(PP)) {  // rare, quad-uniform: P = Q or P = -Q
    const bool inf = rr_is_zero_prod(PP);
    const bool dbl = inf && rr_is_zero_prod(RR);
    XYZZ<F> d = xyzz_zero<F>();
    if (dbl) d = rr_dbl_x4(p);
    rr_sel(o, inf, d);
  }
  return o;
}

// lane-pair forms exist for the reduced-radix G1 points (and, curve_rr2.hpp,
// G2); quads for G1
template <class PF>
struct PairOps {
  static constexpr bool ok = false;
};
template <class Q>
struct PairOps<FpR<Q>> {
  static constexpr bool ok = true;
};
template <class PF>
struct QuadOps {
  static constexpr bool ok = false;
};
template <class Q>
struct QuadOps<FpR<Q>> {
  static constexpr bool ok = true;
};

// ---------------------------------------------------------------------------
// point-arithmetic policy used by the MSM kernels (msm_impl.hpp): one name per
// operation, overloaded on the coordinate field -- the 32-bit-limb lazy
// formulas of curve.hpp (G2 over Fq2, A/B) or the reduced-radix ones above.
// ---------------------------------------------------------------------------
template <class F>
ECG_DEV XYZZ<F> pa_add_affine(const XYZZ<F>& p, const Affine<F>& a) {
  return xyzz_add_affine<F, true>(p, a);
}
template <class Q>
ECG_DEV XYZZ<FpR<Q>> pa_add_affine(const XYZZ<FpR<Q>>& p, const Affine<FpR<Q>>& a) {
  return rr_add_affine(p, a);
}

template <class F>
ECG_DEV XYZZ<F> pa_add(const XYZZ<F>& p, const XYZZ<F>& q) {
  return xyzz_add<F, true>(p, q);
}
template <class Q>
ECG_DEV XYZZ<FpR<Q>> pa_add(const XYZZ<FpR<Q>>& p, const XYZZ<FpR<Q>>& q) {
  return rr_add_xyzz(p, q);
}

template <class F>
ECG_DEV XYZZ<F> pa_dbl(const XYZZ<F>& p) {
  return xyzz_dbl<F, true>(p);
}
template <class Q>
ECG_DEV XYZZ<FpR<Q>> pa_dbl(const XYZZ<FpR<Q>>& p) {
  return rr_dbl(p);
}

// Point operations of latency-bound chains: one lane per operation (PM = 0),
// a lane pair (lanes ^ PM, PM = 1 or 2) or a quad (PM = 4, lanes & 3)
// sharing each operation's products
template <int PM>
constexpr uint32_t pp_lanes_log() {
  return PM == 0 ? 0u : PM == 4 ? 2u : 1u;
}
template <int PM, class PF>
ECG_DEV XYZZ<PF> pp_dbl(const XYZZ<PF>& p) {
  if constexpr (PM == 4)
    return rr_dbl_x4(p);
  else if constexpr (PM != 0)
    return rr_dbl_x2<PM>(p);
  else
    return pa_dbl(p);
}
template <int PM, class PF>
ECG_DEV XYZZ<PF> pp_add(const XYZZ<PF>& p, const XYZZ<PF>& q) {
  if constexpr (PM == 4)
    return rr_add_x4(p, q);
  else if constexpr (PM != 0)
    return rr_add_x2<PM>(p, q);
  else
    return pa_add(p, q);
}

template <class F>
ECG_DEV bool pa_is_zero(const XYZZ<F>& p) {
  return xyzz_is_zero<F, true>(p);
}
template <class Q>
ECG_DEV bool pa_is_zero(const XYZZ<FpR<Q>>& p) {
  return xyzz_is_zero_rr(p);
}

// -P; the reduced-radix Y becomes 8p - Y (<= 8p): stored-point Y only ever
// enters products (add-2008-s, dbl-2008-s-1), whose inputs have ample slack
template <class F>
ECG_DEV XYZZ<F> pa_neg(const XYZZ<F>& p) {
  return xyzz_neg<F, true>(p);
}
template <class Q>
ECG_DEV XYZZ<FpR<Q>> pa_neg(const XYZZ<FpR<Q>>& p) {
  XYZZ<FpR<Q>> r = p;
  if constexpr (rr_tight<Q>())
    r.Y = rr_reduce_q(rr_neg<4>(p.Y));
  else
    r.Y = rr_neg<8>(p.Y);
  return r;
}

// k P for a canonical 256-bit k (8 x u32), double-and-add from the top bit
template <class F>
ECG_DEV XYZZ<F> pa_mul_scalar(const XYZZ<F>& p, const uint32_t* k) {
  int top = 255;
  while (top >= 0 && !((k[top >> 5] >> (top & 31)) & 1)) top--;
  if (top < 0 || pa_is_zero(p)) return xyzz_zero<F>();
  XYZZ<F> acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = pa_dbl(acc);
    if ((k[b >> 5] >> (b & 31)) & 1) acc = pa_add(acc, p);
  }
  return acc;
}

// lazy 32-bit-limb XYZZ -> the pipeline's coordinate field
template <class F>
ECG_DEV XYZZ<F> pa_from_std(const XYZZ<F>& p) {
  return p;
}
template <class Q>
ECG_DEV XYZZ<FpR<Q>> pa_from_std_rr(const XYZZ<Fp<typename Q::Base>>& p) {
  XYZZ<FpR<Q>> r;
  r.X = rr_from_std<Q>(p.X);
  r.Y = rr_from_std<Q>(p.Y);
  r.ZZ = rr_from_std<Q>(p.ZZ);
  r.ZZZ = rr_from_std<Q>(p.ZZZ);
  return r;
}

// x * c for a boundary-form constant c (the GLV endomorphism's beta)
template <class F>
ECG_DEV F pa_mul_const(const F& x, const F& c) {
  return fmul_lz(x, c);
}
template <class Q>
ECG_DEV FpR<Q> pa_mul_const(const FpR<Q>& x, const Fp<typename Q::Base>& c) {
  return rr_mul(x, rr_from_std<Q>(c));
}

// Coordinate field of the bucket / butterfly pipelines: the reduced-radix
// form for the G1 base fields, the 32-bit-limb lazy form for G2 (Fq2).
template <class FqP>
struct RRof {
  using Q = void;
};
template <>
struct RRof<params::bls12_381_fq> {
  using Q = params::bls12_381_fq_rr;
};
template <>
struct RRof<params::bn254_fq> {
  using Q = params::bn254_fq_rr;
};
// G1 bucket layout: BN254 takes the 9 x 29-bit tight-slack form (fewer mads
// per product); G2's Fq2 keeps RRof's 10 x 28 bits.
template <class FqP>
struct RR1of {
  using Q = typename RRof<FqP>::Q;
};
template <>
struct RR1of<params::bn254_fq> {
  using Q = params::bn254_fq9_rr;
};
// BLS12-381 G1 buckets: 13 x 30 bits (338 instead of 392 mads per product,
// split columns, tight-slack formulas at R'/p ~ 2^9.4); A/B: -DECG_BLS_FQ14
// keeps 14 x 29 bits
#ifndef ECG_BLS_FQ14
template <>
struct RR1of<params::bls12_381_fq> {
  using Q = params::bls12_381_fq13_rr;
};
#endif
template <class C>
constexpr bool has_rr_form() {
  return C::EXT == 1 && !std::is_same<typename RRof<typename C::FqParams>::Q, void>::value;
}

// negated base y (y <= M); the reduced-radix form stays wide (no carry
// step): it only meets product outputs in rr_add_affine
template <class F>
ECG_DEV F pa_neg_y(const F& y) {
  return fneg_lz(y);
}
template <class Q>
ECG_DEV FpR<Q> pa_neg_y(const FpR<Q>& y) {
  if constexpr (Q::BITS > 29)  // 30-bit limbs: wide limbs (< 3 2^30) would overflow the product columns
    return rr_neg<4>(y);
  else
    return rr_neg_wide<4>(y);
}

// k P for a small unsigned k (double-and-add from the MSB)
template <class F>
ECG_DEV XYZZ<F> pa_mul_small(const XYZZ<F>& p, uint32_t k) {
  XYZZ<F> acc = xyzz_zero<F>();
  if (k == 0) return acc;
  const int top = 31 - __builtin_clz(k);
  acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = pa_dbl(acc);
    if ((k >> b) & 1) acc = pa_add(acc, p);
  }
  return acc;
}

// bucket-pipeline point -> lazy 32-bit-limb XYZZ (canonical coordinates)
template <class F>
ECG_DEV XYZZ<F> pa_to_std(const XYZZ<F>& p) {
  return p;
}
template <class Q>
ECG_DEV XYZZ<Fp<typename Q::Base>> pa_to_std(const XYZZ<FpR<Q>>& p) {
  XYZZ<Fp<typename Q::Base>> r;
  if (xyzz_is_zero_rr(p)) return xyzz_zero<Fp<typename Q::Base>>();
  r.X = rr_to_std(p.X);
  r.Y = rr_to_std(p.Y);
  r.ZZ = rr_to_std(p.ZZ);
  r.ZZZ = rr_to_std(p.ZZZ);
  return r;
}

// ---------------------------------------------------------------------------
// memory: a reduced-radix affine base is 2 NL words, an XYZZ point 4 NL words,
// moved as 16-B vectors.  A word count that is not a multiple of 4 (the 9-limb
// BN254 G1 base: 18 words) moves whole vectors: the last one reads / writes
// up to 3 words past the value, which the 128-B base records (BaseLayout)
// leave as padding.
template <int W>
constexpr int rr_vec_words() {
  return (W + 3) / 4 * 4;
}
template <class Q, int W>
ECG_DEV void rr_load_words(const void* src, uint32_t* w) {
  constexpr int V = rr_vec_words<W>();
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int i = 0; i < V / 4; i++) {
    const uint4 t = s[i];
    const uint32_t q[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (4 * i + k < W) w[4 * i + k] = q[k];
  }
}

template <class Q, int W>
ECG_DEV void rr_store_words(void* dst, const uint32_t* w) {
  constexpr int V = rr_vec_words<W>();
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int i = 0; i < V / 4; i++) {
    uint32_t q[4];
#pragma unroll
    for (int k = 0; k < 4; k++) q[k] = 4 * i + k < W ? w[4 * i + k] : 0u;
    d[i] = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

template <class Q>
ECG_DEV Affine<FpR<Q>> load_affine(const FpR<Q>* xy) {
  constexpr int NL = Q::NL;
  uint32_t w[2 * NL];
  rr_load_words<Q, 2 * NL>(xy, w);
  Affine<FpR<Q>> a;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    a.x.v[i] = w[i];
    a.y.v[i] = w[NL + i];
  }
  return a;
}

template <class Q>
ECG_DEV void store_affine(FpR<Q>* xy, const Affine<FpR<Q>>& a) {
  constexpr int NL = Q::NL;
  uint32_t w[2 * NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    w[i] = a.x.v[i];
    w[NL + i] = a.y.v[i];
  }
  rr_store_words<Q, 2 * NL>(xy, w);
}

template <class Q>
ECG_DEV XYZZ<FpR<Q>> load_xyzz(const XYZZ<FpR<Q>>* src) {
  constexpr int NL = Q::NL;
  uint32_t w[4 * NL];
  rr_load_words<Q, 4 * NL>(src, w);
  XYZZ<FpR<Q>> p;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    p.X.v[i] = w[i];
    p.Y.v[i] = w[NL + i];
    p.ZZ.v[i] = w[2 * NL + i];
    p.ZZZ.v[i] = w[3 * NL + i];
  }
  return p;
}

template <class Q>
ECG_DEV void store_xyzz(XYZZ<FpR<Q>>* dst, const XYZZ<FpR<Q>>& p) {
  constexpr int NL = Q::NL;
  uint32_t w[4 * NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    w[i] = p.X.v[i];
    w[NL + i] = p.Y.v[i];
    w[2 * NL + i] = p.ZZ.v[i];
    w[3 * NL + i] = p.ZZZ.v[i];
  }
  rr_store_words<Q, 4 * NL>(dst, w);
}

}  // namespace ecg
