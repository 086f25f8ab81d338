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

// Montgomery CIOS with 64-bit words
template <class P>
static inline HFp<P> hmul(const HFp<P>& a, const HFp<P>& b) {
  constexpr int N = P::N;
  uint64_t t[N + 2] = {0};
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
    for (int j = 0; j < N; j++) {
      u128 x = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    u128 x = (u128)t[N] + c;
    t[N] = (uint64_t)x;
    t[N + 1] = (uint64_t)(x >> 64);
    const uint64_t m = t[0] * P::INV;
    x = (u128)m * P::P[0] + t[0];
    c = (uint64_t)(x >> 64);
    for (int j = 1; j < N; j++) {
      x = (u128)m * P::P[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    x = (u128)t[N] + c;
    t[N - 1] = (uint64_t)x;
    t[N] = t[N + 1] + (uint64_t)(x >> 64);
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

// XYZZ points (x = X/ZZ, y = Y/ZZZ), identity ZZ == 0 -- same formulas as
// the device code in curve.hpp (EFD g1p/auto-shortw-xyzz, a = 0).
template <class P>
struct HXYZZ {
  HFp<P> X, Y, ZZ, ZZZ;
  bool is_zero() const { return ZZ.is_zero(); }
  static HXYZZ zero() { return HXYZZ{HFp<P>::one(), HFp<P>::one(), HFp<P>::zero(), HFp<P>::zero()}; }
};

template <class P>
static inline HXYZZ<P> hdbl(const HXYZZ<P>& p) {
  if (p.is_zero()) return p;
  HFp<P> U = hadd(p.Y, p.Y);
  HFp<P> V = hmul(U, U);
  HFp<P> W = hmul(U, V);
  HFp<P> S = hmul(p.X, V);
  HFp<P> X2 = hmul(p.X, p.X);
  HFp<P> M = hadd(hadd(X2, X2), X2);
  HXYZZ<P> r;
  r.X = hsub(hsub(hmul(M, M), S), S);
  r.Y = hsub(hmul(M, hsub(S, r.X)), hmul(W, p.Y));
  r.ZZ = hmul(V, p.ZZ);
  r.ZZZ = hmul(W, p.ZZZ);
  return r;
}

template <class P>
static inline HXYZZ<P> hadd_pts(const HXYZZ<P>& p, const HXYZZ<P>& q) {
  if (p.is_zero()) return q;
  if (q.is_zero()) return p;
  HFp<P> U1 = hmul(p.X, q.ZZ), U2 = hmul(q.X, p.ZZ);
  HFp<P> S1 = hmul(p.Y, q.ZZZ), S2 = hmul(q.Y, p.ZZZ);
  HFp<P> Pd = hsub(U2, U1), R = hsub(S2, S1);
  if (Pd.is_zero()) {
    if (R.is_zero()) return hdbl(p);
    return HXYZZ<P>::zero();
  }
  HFp<P> PP = hmul(Pd, Pd), PPP = hmul(Pd, PP), Q = hmul(U1, PP);
  HXYZZ<P> r;
  r.X = hsub(hsub(hsub(hmul(R, R), PPP), Q), Q);
  r.Y = hsub(hmul(R, hsub(Q, r.X)), hmul(S1, PPP));
  r.ZZ = hmul(hmul(p.ZZ, q.ZZ), PP);
  r.ZZZ = hmul(hmul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// Jacobian (X, Y, Z) -> XYZZ
template <class P>
static inline HXYZZ<P> hfrom_jac(const uint64_t* j) {
  HXYZZ<P> r;
  HFp<P> Z;
  memcpy(r.X.v, j, sizeof r.X.v);
  memcpy(r.Y.v, j + P::N, sizeof r.Y.v);
  memcpy(Z.v, j + 2 * P::N, sizeof Z.v);
  if (Z.is_zero()) return HXYZZ<P>::zero();
  r.ZZ = hmul(Z, Z);
  r.ZZZ = hmul(r.ZZ, Z);
  return r;
}

// normalised Jacobian (x, y, 1) or (0, 1, 0)
template <class P>
static inline void hto_jac_norm(const HXYZZ<P>& p, uint64_t* out) {
  constexpr int N = P::N;
  if (p.is_zero()) {
    HFp<P> z = HFp<P>::zero(), o = HFp<P>::one();
    memcpy(out, z.v, 8 * N);
    memcpy(out + N, o.v, 8 * N);
    memcpy(out + 2 * N, z.v, 8 * N);
    return;
  }
  HFp<P> inv = hinv(hmul(p.ZZ, p.ZZZ));
  HFp<P> x = hmul(p.X, hmul(inv, p.ZZZ));
  HFp<P> y = hmul(p.Y, hmul(inv, p.ZZ));
  HFp<P> o = HFp<P>::one();
  memcpy(out, x.v, 8 * N);
  memcpy(out + N, y.v, 8 * N);
  memcpy(out + 2 * N, o.v, 8 * N);
}

}  // namespace host
}  // namespace ecg
