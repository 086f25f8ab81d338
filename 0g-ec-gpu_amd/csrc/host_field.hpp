// Host-side (x86) Montgomery arithmetic and XYZZ point ops for the short
// serial tails of the MSM: the Horner fold over window sums and the final
// affine normalisation.  This is the reference GPU path's own split -- the
// GPU returns per-window results and the host folds them (ec-gpu-proxy/src/
// multiexp.rs:221-233, 394-397) -- kept on the host because one serial chain
// of ~256 doublings runs ~25x faster on a CPU core than on one GPU lane
// ("serial tails").  Same representation as the device code:
// N x u64 limbs, R = 2^(64N), fully reduced.
#pragma once
#include <stdint.h>
#include <string.h>

namespace ecg {
namespace host {

typedef unsigned __int128 u128;

template <class P>
struct HFp {
  static constexpr int N = P::N;
  uint64_t v[N];
  static HFp zero() {
    HFp r;
    memset(r.v, 0, sizeof r.v);
    return r;
  }
  static HFp one() {
    HFp r;
    for (int i = 0; i < N; i++) r.v[i] = P::ONE[i];
    return r;
  }
  bool is_zero() const {
    uint64_t o = 0;
    for (int i = 0; i < N; i++) o |= v[i];
    return o == 0;
  }
  bool operator==(const HFp& b) const { return memcmp(v, b.v, sizeof v) == 0; }
};

template <class P>
static inline bool geq_p(const uint64_t* a) {
  for (int i = P::N - 1; i >= 0; i--) {
    if (a[i] != P::P[i]) return a[i] > P::P[i];
  }
  return true;
}

template <class P>
static inline void sub_p(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < P::N; i++) {
    u128 d = (u128)a[i] - P::P[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}

// device lazy range [0, 2p] -> canonical [0, p)
template <class P>
static inline HFp<P> hcanon(HFp<P> a) {
  while (geq_p<P>(a.v)) sub_p<P>(a.v);
  return a;
}

template <class P>
static inline HFp<P> hadd(const HFp<P>& a, const HFp<P>& b) {
  HFp<P> r;
  uint64_t c = 0;
  for (int i = 0; i < P::N; i++) {
    u128 s = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (geq_p<P>(r.v)) sub_p<P>(r.v);
  return r;
}

template <class P>
static inline HFp<P> hsub(const HFp<P>& a, const HFp<P>& b) {
  HFp<P> r;
  uint64_t br = 0;
  for (int i = 0; i < P::N; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < P::N; i++) {
      u128 s = (u128)r.v[i] + P::P[i] + c;
      r.v[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  return r;
}

// Montgomery CIOS with 64-bit words, unrolled; the top word's carry is kept
// as a flag instead of a second 128-bit add (on the host fold's serial
// doubling chains, profiles/r05: ~0.2 ms of a 2^20 MSM is host time)
template <class P>
static inline HFp<P> hmul(const HFp<P>& a, const HFp<P>& b) {
  constexpr int N = P::N;
  uint64_t t[N + 1] = {0};
#pragma GCC unroll 8
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
#pragma GCC unroll 8
    for (int j = 0; j < N; j++) {
      const u128 x = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    const uint64_t tn = t[N] + c;
    const uint64_t hi = tn < c;
    const uint64_t m = t[0] * P::INV;
    u128 x = (u128)m * P::P[0] + t[0];
    c = (uint64_t)(x >> 64);
#pragma GCC unroll 8
    for (int j = 1; j < N; j++) {
      x = (u128)m * P::P[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    x = (u128)tn + c;
    t[N - 1] = (uint64_t)x;
    t[N] = hi + (uint64_t)(x >> 64);
  }
  if (t[N] || geq_p<P>(t)) sub_p<P>(t);
  HFp<P> r;
  memcpy(r.v, t, sizeof r.v);
  return r;
}

template <class P>
static inline HFp<P> hinv(const HFp<P>& a) {  // a^(p-2)
  HFp<P> r = HFp<P>::one();
  for (int i = P::N - 1; i >= 0; i--)
    for (int bit = 63; bit >= 0; bit--) {
      r = hmul(r, r);
      if ((P::PM2[i] >> bit) & 1) r = hmul(r, a);
    }
  return r;
}

// Fq2 = Fq[u]/(u^2 + 1) on the host (G2 folds), c0 then c1 as on the device.
template <class P>
struct HFp2 {
  static constexpr int N = 2 * P::N;  // u64 words
  HFp<P> c0, c1;
  static HFp2 zero() { return HFp2{HFp<P>::zero(), HFp<P>::zero()}; }
  static HFp2 one() { return HFp2{HFp<P>::one(), HFp<P>::zero()}; }
  bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  bool operator==(const HFp2& b) const { return c0 == b.c0 && c1 == b.c1; }
};

template <class P>
static inline HFp2<P> hadd(const HFp2<P>& a, const HFp2<P>& b) {
  return HFp2<P>{hadd(a.c0, b.c0), hadd(a.c1, b.c1)};
}
template <class P>
static inline HFp2<P> hsub(const HFp2<P>& a, const HFp2<P>& b) {
  return HFp2<P>{hsub(a.c0, b.c0), hsub(a.c1, b.c1)};
}
template <class P>
static inline HFp2<P> hmul(const HFp2<P>& a, const HFp2<P>& b) {
  HFp<P> aa = hmul(a.c0, b.c0), bb = hmul(a.c1, b.c1);
  HFp<P> t = hmul(hadd(a.c0, a.c1), hadd(b.c0, b.c1));
  return HFp2<P>{hsub(aa, bb), hsub(hsub(t, aa), bb)};
}
template <class P>
static inline HFp2<P> hinv(const HFp2<P>& a) {
  HFp<P> t = hinv(hadd(hmul(a.c0, a.c0), hmul(a.c1, a.c1)));
  HFp<P> z = HFp<P>::zero();
  return HFp2<P>{hmul(a.c0, t), hsub(z, hmul(a.c1, t))};
}
template <class P>
static inline HFp2<P> hcanon(HFp2<P> a) {
  return HFp2<P>{hcanon(a.c0), hcanon(a.c1)};
}

// XYZZ points (x = X/ZZ, y = Y/ZZZ), identity ZZ == 0 -- same formulas as
// the device code in curve.hpp (EFD g1p/auto-shortw-xyzz, a = 0), over any
// coordinate field HF (HFp for G1, HFp2 for G2).
template <class HF>
struct HPoint {
  HF X, Y, ZZ, ZZZ;
  bool is_zero() const { return ZZ.is_zero(); }
  static HPoint zero() { return HPoint{HF::one(), HF::one(), HF::zero(), HF::zero()}; }
};
template <class P>
using HXYZZ = HPoint<HFp<P>>;

template <class HF>
static inline HPoint<HF> hdbl(const HPoint<HF>& p) {
  if (p.is_zero()) return p;
  HF U = hadd(p.Y, p.Y);
  HF V = hmul(U, U);
  HF W = hmul(U, V);
  HF S = hmul(p.X, V);
  HF X2 = hmul(p.X, p.X);
  HF M = hadd(hadd(X2, X2), X2);
  HPoint<HF> r;
  r.X = hsub(hsub(hmul(M, M), S), S);
  r.Y = hsub(hmul(M, hsub(S, r.X)), hmul(W, p.Y));
  r.ZZ = hmul(V, p.ZZ);
  r.ZZZ = hmul(W, p.ZZZ);
  return r;
}

template <class HF>
static inline HPoint<HF> hadd_pts(const HPoint<HF>& p, const HPoint<HF>& q) {
  if (p.is_zero()) return q;
  if (q.is_zero()) return p;
  HF U1 = hmul(p.X, q.ZZ), U2 = hmul(q.X, p.ZZ);
  HF S1 = hmul(p.Y, q.ZZZ), S2 = hmul(q.Y, p.ZZZ);
  HF Pd = hsub(U2, U1), R = hsub(S2, S1);
  if (Pd.is_zero()) {
    if (R.is_zero()) return hdbl(p);
    return HPoint<HF>::zero();
  }
  HF PP = hmul(Pd, Pd), PPP = hmul(Pd, PP), Q = hmul(U1, PP);
  HPoint<HF> r;
  r.X = hsub(hsub(hsub(hmul(R, R), PPP), Q), Q);
  r.Y = hsub(hmul(R, hsub(Q, r.X)), hmul(S1, PPP));
  r.ZZ = hmul(hmul(p.ZZ, q.ZZ), PP);
  r.ZZZ = hmul(hmul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// Jacobian points (a = 0) for the host's serial doubling chains -- the
// window fold's c (W - 1) doublings: dbl-2009-l is 2M + 5S where the XYZZ
// doubling above is 6M + 3S.  Identity: Z == 0.
template <class HF>
struct HJac {
  HF X, Y, Z;
  bool is_zero() const { return Z.is_zero(); }
  static HJac zero() { return HJac{HF::one(), HF::one(), HF::zero()}; }
};

template <class HF>
static inline HJac<HF> hjac_from_xyzz(const HPoint<HF>& p) {  // (X ZZ ZZZ^2, Y ZZ^3 ZZZ^2, ZZ ZZZ)
  if (p.is_zero()) return HJac<HF>::zero();
  const HF z3sq = hmul(p.ZZZ, p.ZZZ);
  const HF zz3 = hmul(hmul(p.ZZ, p.ZZ), p.ZZ);
  return HJac<HF>{hmul(hmul(p.X, p.ZZ), z3sq), hmul(hmul(p.Y, zz3), z3sq), hmul(p.ZZ, p.ZZZ)};
}

template <class HF>
static inline HPoint<HF> hxyzz_from_jac(const HJac<HF>& j) {
  if (j.is_zero()) return HPoint<HF>::zero();
  const HF zz = hmul(j.Z, j.Z);
  return HPoint<HF>{j.X, j.Y, zz, hmul(zz, j.Z)};
}

template <class HF>
static inline HJac<HF> hjac_dbl(const HJac<HF>& p) {
  if (p.is_zero()) return p;
  const HF A = hmul(p.X, p.X), B = hmul(p.Y, p.Y), C = hmul(B, B);
  const HF xb = hadd(p.X, B);
  HF D = hsub(hsub(hmul(xb, xb), A), C);
  D = hadd(D, D);
  const HF E = hadd(hadd(A, A), A), F = hmul(E, E);
  HJac<HF> r;
  r.X = hsub(hsub(F, D), D);
  HF C8 = hadd(C, C);
  C8 = hadd(C8, C8);
  C8 = hadd(C8, C8);
  r.Y = hsub(hmul(E, hsub(D, r.X)), C8);
  const HF yz = hmul(p.Y, p.Z);
  r.Z = hadd(yz, yz);
  return r;
}

template <class HF>
static inline HJac<HF> hjac_add(const HJac<HF>& p, const HJac<HF>& q) {  // add-2007-bl
  if (p.is_zero()) return q;
  if (q.is_zero()) return p;
  const HF Z1Z1 = hmul(p.Z, p.Z), Z2Z2 = hmul(q.Z, q.Z);
  const HF U1 = hmul(p.X, Z2Z2), U2 = hmul(q.X, Z1Z1);
  const HF S1 = hmul(hmul(p.Y, q.Z), Z2Z2), S2 = hmul(hmul(q.Y, p.Z), Z1Z1);
  const HF H = hsub(U2, U1);
  HF rr = hsub(S2, S1);
  if (H.is_zero()) return rr.is_zero() ? hjac_dbl(p) : HJac<HF>::zero();
  const HF H2 = hadd(H, H), I = hmul(H2, H2), J = hmul(H, I);
  rr = hadd(rr, rr);
  const HF V = hmul(U1, I);
  HJac<HF> r;
  r.X = hsub(hsub(hsub(hmul(rr, rr), J), V), V);
  const HF S1J = hmul(S1, J);
  r.Y = hsub(hmul(rr, hsub(V, r.X)), hadd(S1J, S1J));
  const HF zs = hadd(p.Z, q.Z);
  r.Z = hmul(hsub(hsub(hmul(zs, zs), Z1Z1), Z2Z2), H);
  return r;
}

// Jacobian (X, Y, Z), each coordinate HF::N u64 words -> XYZZ
template <class HF>
static inline HPoint<HF> hfrom_jac_t(const uint64_t* j) {
  constexpr int N = HF::N;
  HPoint<HF> r;
  HF Z;
  memcpy(&r.X, j, 8 * N);
  memcpy(&r.Y, j + N, 8 * N);
  memcpy(&Z, j + 2 * N, 8 * N);
  if (Z.is_zero()) return HPoint<HF>::zero();
  r.ZZ = hmul(Z, Z);
  r.ZZZ = hmul(r.ZZ, Z);
  return r;
}
template <class P>
static inline HXYZZ<P> hfrom_jac(const uint64_t* j) {
  return hfrom_jac_t<HFp<P>>(j);
}

// normalised Jacobian (x, y, 1) or (0, 1, 0)
template <class HF>
static inline void hto_jac_norm(const HPoint<HF>& p, uint64_t* out) {
  constexpr int N = HF::N;
  if (p.is_zero()) {
    HF z = HF::zero(), o = HF::one();
    memcpy(out, &z, 8 * N);
    memcpy(out + N, &o, 8 * N);
    memcpy(out + 2 * N, &z, 8 * N);
    return;
  }
  HF inv = hinv(hmul(p.ZZ, p.ZZZ));
  HF x = hmul(p.X, hmul(inv, p.ZZZ));
  HF y = hmul(p.Y, hmul(inv, p.ZZ));
  HF o = HF::one();
  memcpy(out, &x, 8 * N);
  memcpy(out + N, &y, 8 * N);
  memcpy(out + 2 * N, &o, 8 * N);
}

}  // namespace host
}  // namespace ecg
