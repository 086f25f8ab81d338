// G2 in the reduced-radix form: Fq2 = Fq[u]/(u^2 + 1) over the 29-/28-bit-limb
// Montgomery elements of fieldrr.hpp, and the XYZZ formulas of curve_rr.hpp
// restated over it (madd-2008-s, add-2008-s, dbl-2008-s-1 / mdbl-2008-s-1;
// ec.cl:17-130 and field2.cl:1-61's roles for the MSM bucket pipeline).
//
// An Fq2 product is two one-reduction product sums (rr_mul_sum2):
//   c0 = (a0 b0 + a1 (K p - b1)) / R',  c1 = (a0 b1 + a1 b0) / R'
// -- 4 products and 2 reductions, the same mad count as Karatsuba's 3 + 3 with
// no operand sums; a square is the complex method as one interleaved pair,
//   c0 = (a0 + a1)(a0 - a1 + K p) / R',  c1 = (2 a0) a1 / R'.
// Every output component is a product output (exact limbs, value < p (1 + 2^-9)),
// so the zero screens of curve_rr.hpp work per component.
//
// Bounds (units of p, per component; M = product output):
//   stored points  X <= 17.01, Y <= 4.01, ZZ, ZZZ <= M;  bases x <= M,
//                  y <= M or 4p - y (carried: every G2 product operand is QN)
//   madd:  P = U2 - X1 + 64p <= 65, R = S2 - Y1 + 16p <= 17,
//          X3 = R^2 - PPP - 2Q + 16p <= 17.01, D = Q - X3 + 64p <= 65,
//          Y3 = D R + Y1 (4p - PPP)   (two product outputs summed) <= 2.01
//   add:   P, R <= 5.01, the rest as madd;  dbl: U = 2Y <= 8.02, M = 3X^2 <= 3.01
// The K of each negated operand is at least twice its bound; the largest
// product sum is 130 x 321 p^2 (the square of P), far inside the 2^24 p^2 that
// the 2^25 slack of rr_mul allows.
#pragma once
#include "curve_rr.hpp"
#include "field2.hpp"

namespace ecg {

template <class Q>
struct FpR2 {
  using Params = Q;
  using Base = FpR<Q>;
  FpR<Q> c0, c1;
  ECG_DEV static FpR2 zero() {
    FpR2 r;
    r.c0 = FpR<Q>::zero();
    r.c1 = FpR<Q>::zero();
    return r;
  }
  ECG_DEV static FpR2 one() {
    FpR2 r;
    r.c0 = FpR<Q>::one();
    r.c1 = FpR<Q>::zero();
    return r;
  }
};

template <class Q>
ECG_DEV FpR2<Q> mkr2(const FpR<Q>& a, const FpR<Q>& b) {
  FpR2<Q> r;
  r.c0 = a;
  r.c1 = b;
  return r;
}

// a b; b.c1 <= K p / 2
template <int K, class Q>
ECG_DEV FpR2<Q> r2_mul(const FpR2<Q>& a, const FpR2<Q>& b) {
  return mkr2(rr_mul_sum2(a.c0, b.c0, a.c1, rr_neg<K>(b.c1)), rr_mul_sum2(a.c0, b.c1, a.c1, b.c0));
}
// a^2; a.c1 <= K p / 2
template <int K, class Q>
ECG_DEV FpR2<Q> r2_sqr(const FpR2<Q>& a) {
  FpR2<Q> r;
  rr_mul2(rr_add(a.c0, a.c1), rr_sub<K>(a.c0, a.c1), rr_add(a.c0, a.c0), a.c1, r.c0, r.c1);
  return r;
}
template <class Q>
ECG_DEV FpR2<Q> r2_add(const FpR2<Q>& a, const FpR2<Q>& b) {
  return mkr2(rr_add(a.c0, b.c0), rr_add(a.c1, b.c1));
}
template <int K, class Q>
ECG_DEV FpR2<Q> r2_sub(const FpR2<Q>& a, const FpR2<Q>& b) {
  return mkr2(rr_sub<K>(a.c0, b.c0), rr_sub<K>(a.c1, b.c1));
}
template <int K, class Q>
ECG_DEV FpR2<Q> r2_sub2(const FpR2<Q>& a, const FpR2<Q>& b, const FpR2<Q>& c) {
  return mkr2(rr_sub2<K>(a.c0, b.c0, c.c0), rr_sub2<K>(a.c1, b.c1, c.c1));
}
template <int K, class Q>
ECG_DEV FpR2<Q> r2_sub3(const FpR2<Q>& a, const FpR2<Q>& b, const FpR2<Q>& c, const FpR2<Q>& d) {
  return mkr2(rr_sub3<K>(a.c0, b.c0, c.c0, d.c0), rr_sub3<K>(a.c1, b.c1, c.c1, d.c1));
}
template <int K, class Q>
ECG_DEV FpR2<Q> r2_neg(const FpR2<Q>& a) {
  return mkr2(rr_neg<K>(a.c0), rr_neg<K>(a.c1));
}
template <class Q>
ECG_DEV bool fis_zero(const FpR2<Q>& a) {
  return fis_zero(a.c0) && fis_zero(a.c1);
}
template <class Q>
ECG_DEV bool r2_is_zero_prod(const FpR2<Q>& a) {
  return rr_is_zero_prod(a.c0) && rr_is_zero_prod(a.c1);
}
template <class Q>
ECG_DEV bool r2_maybe_zero_prod(const FpR2<Q>& a) {
  return rr_maybe_zero_prod(a.c0) && rr_maybe_zero_prod(a.c1);
}
template <class Q>
ECG_DEV void rr_sel(FpR2<Q>& r, bool c, const FpR2<Q>& s) {
  rr_sel(r.c0, c, s.c0);
  rr_sel(r.c1, c, s.c1);
}
template <class Q>
ECG_DEV void rr_sel(XYZZ<FpR2<Q>>& r, bool c, const XYZZ<FpR2<Q>>& s) {
  rr_sel(r.X, c, s.X);
  rr_sel(r.Y, c, s.Y);
  rr_sel(r.ZZ, c, s.ZZ);
  rr_sel(r.ZZZ, c, s.ZZZ);
}

// ark-ff Fq2 (c0, c1 Montgomery, < p) <-> the reduced-radix form
template <class Q>
ECG_DEV FpR2<Q> rr2_from_std(const Fp2<typename Q::Base>& a) {
  return mkr2(rr_from_std<Q>(a.c0), rr_from_std<Q>(a.c1));
}
template <class Q>
ECG_DEV Fp2<typename Q::Base> rr2_to_std(const FpR2<Q>& a) {
  return mk2(rr_to_std(a.c0), rr_to_std(a.c1));
}

// ---------------------------------------------------------------------------
// XYZZ formulas (the bounds in the header)
// ---------------------------------------------------------------------------
// dbl-2008-s-1 core on (X, Y): new X, Y and the ZZ, ZZZ factors V = U^2, W = U V
template <class Q>
ECG_DEV void r2_dbl_core(const FpR2<Q>& X, const FpR2<Q>& Y, XYZZ<FpR2<Q>>& r, FpR2<Q>& V, FpR2<Q>& W) {
  const FpR2<Q> U = r2_add(Y, Y);
  V = r2_sqr<64>(U);
  const FpR2<Q> X2 = r2_sqr<64>(X);
  W = r2_mul<4>(U, V);
  const FpR2<Q> S = r2_mul<4>(X, V);
  const FpR2<Q> Mm = r2_add(r2_add(X2, X2), X2);
  r.X = r2_sub2<16>(r2_sqr<8>(Mm), S, S);
  r.Y = r2_add(r2_mul<8>(r2_sub<64>(S, r.X), Mm), r2_mul<8>(Y, r2_neg<4>(W)));
}

template <class Q>
ECG_DEV XYZZ<FpR2<Q>> r2_dbl_affine(const Affine<FpR2<Q>>& a) {
  XYZZ<FpR2<Q>> r;
  r2_dbl_core(a.x, a.y, r, r.ZZ, r.ZZZ);
  return r;
}

template <class Q>
ECG_DEV XYZZ<FpR2<Q>> r2_dbl(const XYZZ<FpR2<Q>>& p) {
  if (fis_zero(p.ZZ)) return p;
  XYZZ<FpR2<Q>> r;
  FpR2<Q> V, W;
  r2_dbl_core(p.X, p.Y, r, V, W);
  r.ZZ = r2_mul<4>(p.ZZ, V);
  r.ZZZ = r2_mul<4>(p.ZZZ, W);
  return r;
}

// madd-2008-s: P + (x2, y2); a must not be the identity; a.y QN (<= 4p)
template <class Q>
ECG_DEV XYZZ<FpR2<Q>> r2_add_affine(const XYZZ<FpR2<Q>>& p, const Affine<FpR2<Q>>& a) {
  using F = FpR2<Q>;
  XYZZ<F> r;
  if (fis_zero(p.ZZ)) {
    r.X = a.x;
    r.Y = a.y;
    r.ZZ = F::one();
    r.ZZZ = F::one();
  } else {
    const F U2 = r2_mul<4>(a.x, p.ZZ);
    const F S2 = r2_mul<4>(a.y, p.ZZZ);
    const F P = r2_sub<64>(U2, p.X);
    const F R = r2_sub<16>(S2, p.Y);
    const F PP = r2_sqr<256>(P);
    const F RR = r2_sqr<64>(R);
    const F PPP = r2_mul<4>(P, PP);
    const F Qv = r2_mul<4>(p.X, PP);
    r.ZZ = r2_mul<4>(p.ZZ, PP);
    r.ZZZ = r2_mul<4>(p.ZZZ, PPP);
    r.X = r2_sub3<16>(RR, PPP, Qv, Qv);
    r.Y = r2_add(r2_mul<64>(r2_sub<64>(Qv, r.X), R), r2_mul<8>(p.Y, r2_neg<4>(PPP)));
    if (r2_maybe_zero_prod(PP)) {  // rare: P = Q or P = -Q
      const bool inf = r2_is_zero_prod(PP);
      const bool dbl = inf && r2_is_zero_prod(RR);
      XYZZ<F> d = xyzz_zero<F>();
      if (dbl) d = r2_dbl_affine(a);
      rr_sel(r, inf, d);
    }
  }
  return r;
}

// add-2008-s: P + Q
template <class Q>
ECG_DEV XYZZ<FpR2<Q>> r2_add_xyzz(const XYZZ<FpR2<Q>>& p, const XYZZ<FpR2<Q>>& q) {
  using F = FpR2<Q>;
  const bool pz = fis_zero(p.ZZ), qz = fis_zero(q.ZZ);
  XYZZ<F> r;
  if (pz || qz) {  // single exit, limb selects (see rr_sel)
    r = q;
    rr_sel(r, qz, p);
  } else {
    const F U1 = r2_mul<4>(p.X, q.ZZ);
    const F U2 = r2_mul<4>(q.X, p.ZZ);
    const F S1 = r2_mul<4>(p.Y, q.ZZZ);
    const F S2 = r2_mul<4>(q.Y, p.ZZZ);
    const F P = r2_sub<4>(U2, U1);
    const F R = r2_sub<4>(S2, S1);
    const F PP = r2_sqr<16>(P);
    const F RR = r2_sqr<16>(R);
    const F PPP = r2_mul<4>(P, PP);
    const F Qv = r2_mul<4>(U1, PP);
    r.ZZ = r2_mul<4>(r2_mul<4>(p.ZZ, q.ZZ), PP);
    r.ZZZ = r2_mul<4>(r2_mul<4>(p.ZZZ, q.ZZZ), PPP);
    r.X = r2_sub3<16>(RR, PPP, Qv, Qv);
    r.Y = r2_add(r2_mul<16>(r2_sub<64>(Qv, r.X), R), r2_mul<8>(S1, r2_neg<4>(PPP)));
    if (r2_maybe_zero_prod(PP)) {
      const bool inf = r2_is_zero_prod(PP);
      const bool dbl = inf && r2_is_zero_prod(RR);
      XYZZ<F> d = xyzz_zero<F>();
      if (dbl) d = r2_dbl(p);
      rr_sel(r, inf, d);
    }
  }
  return r;
}

// ---------------------------------------------------------------------------
// Lane-pair forms (curve_rr.hpp rr_dbl_x2's role for G2): every Fq2 product
// is two independent component product sums, so each lane of the pair
// (lanes ^ M) computes one component -- lo c0, hi c1 -- and the pair swaps
// them.  Same formulas, values and bounds as r2_dbl / r2_add_xyzz; half the
// product instructions per lane.  Pair-uniform control flow.
// ---------------------------------------------------------------------------
template <int M, class Q>
ECG_DEV FpR2<Q> r2_join(const FpR<Q>& mine) {  // (c0, c1) from each lane's component
  const bool h = pair_hi<M>();
  const FpR<Q> other = rr_lane_swap<M>(mine);
  return mkr2(rr_pick(h, other, mine), rr_pick(h, mine, other));
}
template <int M, int K, class Q>
ECG_DEV FpR2<Q> r2_mul_x2(const FpR2<Q>& a, const FpR2<Q>& b) {
  const bool h = pair_hi<M>();
  return r2_join<M>(rr_mul_sum2(a.c0, rr_pick(h, b.c1, b.c0), a.c1, rr_pick(h, b.c0, rr_neg<K>(b.c1))));
}
template <int M, int K, class Q>
ECG_DEV FpR2<Q> r2_sqr_x2(const FpR2<Q>& a) {
  const bool h = pair_hi<M>();
  return r2_join<M>(rr_mul(rr_pick(h, rr_add(a.c0, a.c0), rr_add(a.c0, a.c1)), rr_pick(h, a.c1, rr_sub<K>(a.c0, a.c1))));
}

template <int M, class Q>
ECG_DEV XYZZ<FpR2<Q>> rr_dbl_x2(const XYZZ<FpR2<Q>>& p) {
  using F = FpR2<Q>;
  if (fis_zero(p.ZZ)) return p;
  XYZZ<F> r;
  const F U = r2_add(p.Y, p.Y);
  const F V = r2_sqr_x2<M, 64>(U);
  const F X2 = r2_sqr_x2<M, 64>(p.X);
  const F W = r2_mul_x2<M, 4>(U, V);
  const F S = r2_mul_x2<M, 4>(p.X, V);
  const F Mm = r2_add(r2_add(X2, X2), X2);
  r.X = r2_sub2<16>(r2_sqr_x2<M, 8>(Mm), S, S);
  r.Y = r2_add(r2_mul_x2<M, 8>(r2_sub<64>(S, r.X), Mm), r2_mul_x2<M, 8>(p.Y, r2_neg<4>(W)));
  r.ZZ = r2_mul_x2<M, 4>(p.ZZ, V);
  r.ZZZ = r2_mul_x2<M, 4>(p.ZZZ, W);
  return r;
}

template <int M, class Q>
ECG_DEV XYZZ<FpR2<Q>> rr_add_x2(const XYZZ<FpR2<Q>>& p, const XYZZ<FpR2<Q>>& q) {
  using F = FpR2<Q>;
  const bool pz = fis_zero(p.ZZ), qz = fis_zero(q.ZZ);
  XYZZ<F> r;
  if (pz || qz) {
    r = q;
    rr_sel(r, qz, p);
    return r;
  }
  const F U1 = r2_mul_x2<M, 4>(p.X, q.ZZ);
  const F U2 = r2_mul_x2<M, 4>(q.X, p.ZZ);
  const F S1 = r2_mul_x2<M, 4>(p.Y, q.ZZZ);
  const F S2 = r2_mul_x2<M, 4>(q.Y, p.ZZZ);
  const F P = r2_sub<4>(U2, U1);
  const F R = r2_sub<4>(S2, S1);
  const F PP = r2_sqr_x2<M, 16>(P);
  const F RR = r2_sqr_x2<M, 16>(R);
  const F PPP = r2_mul_x2<M, 4>(P, PP);
  const F Qv = r2_mul_x2<M, 4>(U1, PP);
  r.ZZ = r2_mul_x2<M, 4>(r2_mul_x2<M, 4>(p.ZZ, q.ZZ), PP);
  r.ZZZ = r2_mul_x2<M, 4>(r2_mul_x2<M, 4>(p.ZZZ, q.ZZZ), PPP);
  r.X = r2_sub3<16>(RR, PPP, Qv, Qv);
  r.Y = r2_add(r2_mul_x2<M, 16>(r2_sub<64>(Qv, r.X), R), r2_mul_x2<M, 8>(S1, r2_neg<4>(PPP)));
  if (r2_maybe_zero_prod(PP)) {  // pair-uniform: both lanes hold PP, RR
    const bool inf = r2_is_zero_prod(PP);
    const bool dbl = inf && r2_is_zero_prod(RR);
    XYZZ<F> d = xyzz_zero<F>();
    if (dbl) d = rr_dbl_x2<M>(p);
    rr_sel(r, inf, d);
  }
  return r;
}

// Quad forms for G2: lane bit 0 splits each Fq2 product's components (as
// the pair forms above), lane bit 1 splits each level's products (as
// curve_rr.hpp rr_dbl_x2<2> / rr_add_x2<2> on G1).  Each lane computes at most
// two component product sums per level.  Same values and bounds as r2_dbl /
// r2_add_xyzz (a square runs as a product; K is the larger of the two lanes'
// negation bounds, well inside the 2^25 slack).  Quad-uniform control flow.
template <int M, class Q>
ECG_DEV FpR2<Q> r2_lane_swap(const FpR2<Q>& a) {
  return mkr2(rr_lane_swap<M>(a.c0), rr_lane_swap<M>(a.c1));
}
template <class Q>
ECG_DEV FpR2<Q> r2_pick(bool c, const FpR2<Q>& a, const FpR2<Q>& b) {
  return mkr2(rr_pick(c, a.c0, b.c0), rr_pick(c, a.c1, b.c1));
}

template <class Q>
ECG_DEV XYZZ<FpR2<Q>> rr_dbl_x4(const XYZZ<FpR2<Q>>& p) {
  using F = FpR2<Q>;
  if (fis_zero(p.ZZ)) return p;
  const bool h = pair_hi<2>();  // level role; the component role is bit 0
  const F z = F::zero();
  const F U = r2_add(p.Y, p.Y);
  const F L1 = r2_mul_x2<1, 64>(r2_pick(h, p.X, U), r2_pick(h, p.X, U));  // lo V = U^2 | hi X2 = X^2
  const F O1 = r2_lane_swap<2>(L1);
  const F V = r2_pick(h, O1, L1), X2 = r2_pick(h, L1, O1);
  const F Mm = r2_add(r2_add(X2, X2), X2);
  const F a0 = r2_mul_x2<1, 4>(r2_pick(h, p.X, U), V);               // lo W = U V   | hi S = X V
  const F a1 = r2_mul_x2<1, 8>(r2_pick(h, Mm, p.ZZ), r2_pick(h, Mm, V));  // lo ZZ3 = ZZ V | hi M^2
  const F O2 = r2_lane_swap<2>(a0);
  const F W = r2_pick(h, O2, a0), S = r2_pick(h, a0, O2);
  const F X3 = r2_sub2<16>(a1, S, S);  // meaningful on the hi lanes
  const F D = r2_sub<64>(S, X3);
  // lo: ZZZ3 = ZZZ W | hi: Y3 = D M + Y (4p - W)
  const F r = r2_add(r2_mul_x2<1, 8>(r2_pick(h, D, p.ZZZ), r2_pick(h, Mm, W)),
                     r2_mul_x2<1, 8>(r2_pick(h, p.Y, z), r2_pick(h, r2_neg<4>(W), z)));
  const F f = r2_lane_swap<2>(r);                   // lo <- Y3, hi <- ZZZ3
  const F g = r2_lane_swap<2>(r2_pick(h, X3, a1));  // lo <- X3, hi <- ZZ3
  XYZZ<F> o;
  o.X = r2_pick(h, X3, g);
  o.Y = r2_pick(h, r, f);
  o.ZZ = r2_pick(h, g, a1);
  o.ZZZ = r2_pick(h, f, r);
  return o;
}

template <class Q>
ECG_DEV XYZZ<FpR2<Q>> rr_add_x4(const XYZZ<FpR2<Q>>& p, const XYZZ<FpR2<Q>>& q) {
  using F = FpR2<Q>;
  const bool pz = fis_zero(p.ZZ), qz = fis_zero(q.ZZ);
  XYZZ<F> o;
  if (pz || qz) {
    o = q;
    rr_sel(o, qz, p);
    return o;
  }
  const bool h = pair_hi<2>();
  const F z = F::zero();
  const F a0 = r2_mul_x2<1, 4>(r2_pick(h, q.X, p.X), r2_pick(h, p.ZZ, q.ZZ));    // lo U1 | hi U2
  const F a1 = r2_mul_x2<1, 4>(r2_pick(h, q.Y, p.Y), r2_pick(h, p.ZZZ, q.ZZZ));  // lo S1 | hi S2
  const F e0 = r2_lane_swap<2>(a0), e1 = r2_lane_swap<2>(a1);
  const F U1 = r2_pick(h, e0, a0), U2 = r2_pick(h, a0, e0);
  const F S1 = r2_pick(h, e1, a1), S2 = r2_pick(h, a1, e1);
  const F P = r2_sub<4>(U2, U1);
  const F R = r2_sub<4>(S2, S1);
  const F b0 = r2_mul_x2<1, 16>(r2_pick(h, p.ZZ, P), r2_pick(h, q.ZZ, P));    // lo PP | hi ZZ12
  const F b1 = r2_mul_x2<1, 16>(r2_pick(h, p.ZZZ, R), r2_pick(h, q.ZZZ, R));  // lo RR | hi ZZZ12
  const F e2 = r2_lane_swap<2>(b0);
  const F PP = r2_pick(h, e2, b0), ZZ12 = r2_pick(h, b0, e2);
  const F c0 = r2_mul_x2<1, 4>(r2_pick(h, ZZ12, P), PP);   // lo PPP | hi ZZ3
  const F c1 = r2_mul_x2<1, 4>(r2_pick(h, ZZ12, U1), PP);  // lo Q   | hi ZZ3
  const F e3 = r2_lane_swap<2>(c0);
  const F PPP = r2_pick(h, e3, c0), ZZ3 = r2_pick(h, c0, e3);
  const F X3 = r2_sub3<16>(b1, PPP, c1, c1);  // meaningful on the lo lanes
  const F D = r2_sub<64>(c1, X3);
  // lo: Y3 = D R + S1 (4p - PPP) | hi: ZZZ3 = ZZZ12 PPP
  const F r = r2_add(r2_mul_x2<1, 16>(r2_pick(h, b1, D), r2_pick(h, PPP, R)),
                     r2_mul_x2<1, 8>(r2_pick(h, z, S1), r2_pick(h, z, r2_neg<4>(PPP))));
  const F f = r2_lane_swap<2>(r);   // lo <- ZZZ3, hi <- Y3
  const F g = r2_lane_swap<2>(X3);  // hi <- X3
  o.X = r2_pick(h, g, X3);
  o.Y = r2_pick(h, f, r);
  o.ZZ = ZZ3;
  o.ZZZ = r2_pick(h, r, f);
  if (r2_maybe_zero_prod(PP)) {  // rare, quad-uniform (every lane holds PP)
    const F RRv = r2_pick(h, r2_lane_swap<2>(b1), b1);
    const bool inf = r2_is_zero_prod(PP);
    const bool dbl = inf && r2_is_zero_prod(RRv);
    XYZZ<F> d = xyzz_zero<F>();
    if (dbl) d = rr_dbl_x4(p);
    rr_sel(o, inf, d);
  }
  return o;
}

template <class Q>
struct QuadOps<FpR2<Q>> {
  static constexpr bool ok = true;
};

template <class Q>
struct PairOps<FpR2<Q>> {
  static constexpr bool ok = true;
};

// ---------------------------------------------------------------------------
// point-arithmetic policy (curve_rr.hpp) for the Fq2 form
// ---------------------------------------------------------------------------
template <class Q>
ECG_DEV XYZZ<FpR2<Q>> pa_add_affine(const XYZZ<FpR2<Q>>& p, const Affine<FpR2<Q>>& a) {
  return r2_add_affine(p, a);
}
template <class Q>
ECG_DEV XYZZ<FpR2<Q>> pa_add(const XYZZ<FpR2<Q>>& p, const XYZZ<FpR2<Q>>& q) {
  return r2_add_xyzz(p, q);
}
template <class Q>
ECG_DEV XYZZ<FpR2<Q>> pa_dbl(const XYZZ<FpR2<Q>>& p) {
  return r2_dbl(p);
}
template <class Q>
ECG_DEV bool pa_is_zero(const XYZZ<FpR2<Q>>& p) {
  return fis_zero(p.ZZ);
}
// -P: Y becomes 8p - Y (stored Y <= 4p; a negated Y <= 8p only meets
// add-2008-s / dbl-2008-s-1 operands, whose K have the room)
template <class Q>
ECG_DEV XYZZ<FpR2<Q>> pa_neg(const XYZZ<FpR2<Q>>& p) {
  XYZZ<FpR2<Q>> r = p;
  r.Y = r2_neg<8>(p.Y);
  return r;
}
// negated base y, carried (QN): G2 products take no wide operand
template <class Q>
ECG_DEV FpR2<Q> pa_neg_y(const FpR2<Q>& y) {
  return r2_neg<4>(y);
}
template <class Q>
ECG_DEV XYZZ<Fp2<typename Q::Base>> pa_to_std(const XYZZ<FpR2<Q>>& p) {
  if (fis_zero(p.ZZ)) return xyzz_zero<Fp2<typename Q::Base>>();
  XYZZ<Fp2<typename Q::Base>> r;
  r.X = rr2_to_std(p.X);
  r.Y = rr2_to_std(p.Y);
  r.ZZ = rr2_to_std(p.ZZ);
  r.ZZZ = rr2_to_std(p.ZZZ);
  return r;
}

// Coordinate field of the G2 bucket pipeline
template <class C>
constexpr bool has_rr2_form() {
  return C::EXT == 2 && !std::is_same<typename RRof<typename C::FqParams>::Q, void>::value;
}

// ---------------------------------------------------------------------------
// memory: an affine base is 4 NL words, an XYZZ point 8 NL words (16-B moves)
// ---------------------------------------------------------------------------
template <class Q>
ECG_DEV Affine<FpR2<Q>> load_affine(const FpR2<Q>* xy) {
  constexpr int NL = Q::NL;
  uint32_t w[4 * NL];
  rr_load_words<Q, 4 * NL>(xy, w);
  Affine<FpR2<Q>> a;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    a.x.c0.v[i] = w[i];
    a.x.c1.v[i] = w[NL + i];
    a.y.c0.v[i] = w[2 * NL + i];
    a.y.c1.v[i] = w[3 * NL + i];
  }
  return a;
}

template <class Q>
ECG_DEV void store_affine(FpR2<Q>* xy, const Affine<FpR2<Q>>& a) {
  constexpr int NL = Q::NL;
  uint32_t w[4 * NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    w[i] = a.x.c0.v[i];
    w[NL + i] = a.x.c1.v[i];
    w[2 * NL + i] = a.y.c0.v[i];
    w[3 * NL + i] = a.y.c1.v[i];
  }
  rr_store_words<Q, 4 * NL>(xy, w);
}

template <class Q>
ECG_DEV void rr_get_words(FpR<Q>& a, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < Q::NL; i++) a.v[i] = w[i];
}
template <class Q>
ECG_DEV void rr_put_words(uint32_t* w, const FpR<Q>& a) {
#pragma unroll
  for (int i = 0; i < Q::NL; i++) w[i] = a.v[i];
}

template <class Q>
ECG_DEV XYZZ<FpR2<Q>> load_xyzz(const XYZZ<FpR2<Q>>* src) {
  constexpr int NL = Q::NL;
  uint32_t w[8 * NL];
  rr_load_words<Q, 8 * NL>(src, w);
  XYZZ<FpR2<Q>> p;
  rr_get_words(p.X.c0, w);
  rr_get_words(p.X.c1, w + NL);
  rr_get_words(p.Y.c0, w + 2 * NL);
  rr_get_words(p.Y.c1, w + 3 * NL);
  rr_get_words(p.ZZ.c0, w + 4 * NL);
  rr_get_words(p.ZZ.c1, w + 5 * NL);
  rr_get_words(p.ZZZ.c0, w + 6 * NL);
  rr_get_words(p.ZZZ.c1, w + 7 * NL);
  return p;
}

template <class Q>
ECG_DEV void store_xyzz(XYZZ<FpR2<Q>>* dst, const XYZZ<FpR2<Q>>& p) {
  constexpr int NL = Q::NL;
  uint32_t w[8 * NL];
  rr_put_words(w, p.X.c0);
  rr_put_words(w + NL, p.X.c1);
  rr_put_words(w + 2 * NL, p.Y.c0);
  rr_put_words(w + 3 * NL, p.Y.c1);
  rr_put_words(w + 4 * NL, p.ZZ.c0);
  rr_put_words(w + 5 * NL, p.ZZ.c1);
  rr_put_words(w + 6 * NL, p.ZZZ.c0);
  rr_put_words(w + 7 * NL, p.ZZZ.c1);
  rr_store_words<Q, 8 * NL>(dst, w);
}

}  // namespace ecg
