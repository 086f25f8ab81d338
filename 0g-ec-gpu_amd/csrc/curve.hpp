// Short-Weierstrass G1 arithmetic (a = 0) over Fq for gfx950.
//
// Replaces ag-build/cl/ec.cl (POINT_double/add_mixed/add/affine_neg,
// :17-134).  The reference accumulates buckets in Jacobian coordinates
// (madd-2007-bl 7M+4S).  Here buckets use extended-Jacobian "XYZZ"
// coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): mixed add madd-2008-s is
// 8M+2S and needs no squaring of Z -- the cheapest exception-complete-enough
// form for bucket accumulation.  The *value* of every sum is
// the same group element, and outputs are normalised to affine, so results
// are bit-identical to the reference's multiexp_cpu after into_affine()
// (ec-gpu-proxy/tests/multiexp.rs:99).
//
// Identity: ZZ == 0 (XYZZ), Z == 0 (Jacobian, as ec.cl's POINT_ZERO=(0,1,0)),
// and the all-zero affine pair (ag-types/src/impls.rs:52-54 GpuRepr).
#pragma once
#include "field.hpp"

namespace ecg {

template <class FqP, class FrP, class GenP>
struct CurveCfg {
  using Fq = Fp<FqP>;
  using Fr = Fp<FrP>;
  using FqParams = FqP;
  using FrParams = FrP;
  using Gen = GenP;
};

using BLS12_381 = CurveCfg<params::bls12_381_fq, params::bls12_381_fr, params::bls12_381_g1>;
using BN254 = CurveCfg<params::bn254_fq, params::bn254_fr, params::bn254_g1>;

template <class F>
struct Affine {
  F x, y;
};

template <class F>
struct XYZZ {
  F X, Y, ZZ, ZZZ;
};

template <class F>
struct Jac {
  F X, Y, Z;
};

template <class F>
ECG_DEV bool aff_is_identity(const Affine<F>& p) {
  return fis_zero(p.x) && fis_zero(p.y);
}

template <class F>
ECG_DEV XYZZ<F> xyzz_zero() {
  XYZZ<F> r;
  r.X = F::one();
  r.Y = F::one();
  r.ZZ = F::zero();
  r.ZZZ = F::zero();
  return r;
}

template <class F>
ECG_DEV bool xyzz_is_zero(const XYZZ<F>& p) {
  return fis_zero(p.ZZ);
}

template <class F>
ECG_DEV XYZZ<F> xyzz_from_affine(const Affine<F>& a) {
  XYZZ<F> r;
  r.X = a.x;
  r.Y = a.y;
  r.ZZ = F::one();
  r.ZZZ = F::one();
  return r;
}

// mdbl-2008-s-1 (affine input, a = 0): 2 * (x, y)
template <class F>
ECG_DEV XYZZ<F> xyzz_dbl_affine(const Affine<F>& a) {
  F U = fdbl(a.y);
  F V = fsqr(U);
  F W = fmul(U, V);
  F S = fmul(a.x, V);
  F X2 = fsqr(a.x);
  F M = fadd(fdbl(X2), X2);
  XYZZ<F> r;
  r.X = fsub(fsub(fsqr(M), S), S);
  r.Y = fsub(fmul(M, fsub(S, r.X)), fmul(W, a.y));
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// dbl-2008-s-1 (a = 0): 2 * P
template <class F>
ECG_DEV XYZZ<F> xyzz_dbl(const XYZZ<F>& p) {
  if (xyzz_is_zero(p)) return p;
  F U = fdbl(p.Y);
  F V = fsqr(U);
  F W = fmul(U, V);
  F S = fmul(p.X, V);
  F X2 = fsqr(p.X);
  F M = fadd(fdbl(X2), X2);
  XYZZ<F> r;
  r.X = fsub(fsub(fsqr(M), S), S);
  r.Y = fsub(fmul(M, fsub(S, r.X)), fmul(W, p.Y));
  r.ZZ = fmul(V, p.ZZ);
  r.ZZZ = fmul(W, p.ZZZ);
  return r;
}

// madd-2008-s: P + (x2, y2) with y2 optionally negated (signed bucket digit).
// Handles P = O, P = Q (doubling) and P = -Q (identity).  `a` must not be the
// identity (callers skip identity bases).
template <class F>
ECG_DEV XYZZ<F> xyzz_add_affine(const XYZZ<F>& p, const Affine<F>& a) {
  if (xyzz_is_zero(p)) return xyzz_from_affine(a);
  F U2 = fmul(a.x, p.ZZ);
  F S2 = fmul(a.y, p.ZZZ);
  F P = fsub(U2, p.X);
  F R = fsub(S2, p.Y);
  if (fis_zero(P)) {
    if (fis_zero(R)) return xyzz_dbl_affine(a);
    return xyzz_zero<F>();
  }
  F PP = fsqr(P);
  F PPP = fmul(P, PP);
  F Q = fmul(p.X, PP);
  XYZZ<F> r;
  r.X = fsub(fsub(fsub(fsqr(R), PPP), Q), Q);
  r.Y = fsub(fmul(R, fsub(Q, r.X)), fmul(p.Y, PPP));
  r.ZZ = fmul(p.ZZ, PP);
  r.ZZZ = fmul(p.ZZZ, PPP);
  return r;
}

// add-2008-s: P + Q, both XYZZ.
template <class F>
ECG_DEV XYZZ<F> xyzz_add(const XYZZ<F>& p, const XYZZ<F>& q) {
  if (xyzz_is_zero(p)) return q;
  if (xyzz_is_zero(q)) return p;
  F U1 = fmul(p.X, q.ZZ);
  F U2 = fmul(q.X, p.ZZ);
  F S1 = fmul(p.Y, q.ZZZ);
  F S2 = fmul(q.Y, p.ZZZ);
  F P = fsub(U2, U1);
  F R = fsub(S2, S1);
  if (fis_zero(P)) {
    if (fis_zero(R)) return xyzz_dbl(p);
    return xyzz_zero<F>();
  }
  F PP = fsqr(P);
  F PPP = fmul(P, PP);
  F Q = fmul(U1, PP);
  XYZZ<F> r;
  r.X = fsub(fsub(fsub(fsqr(R), PPP), Q), Q);
  r.Y = fsub(fmul(R, fsub(Q, r.X)), fmul(S1, PPP));
  r.ZZ = fmul(fmul(p.ZZ, q.ZZ), PP);
  r.ZZZ = fmul(fmul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

template <class F>
ECG_DEV XYZZ<F> xyzz_neg(const XYZZ<F>& p) {
  XYZZ<F> r = p;
  r.Y = fneg(p.Y);
  return r;
}

// k * P for a small unsigned scalar (double-and-add from the MSB).
template <class F>
ECG_DEV XYZZ<F> xyzz_mul_small(const XYZZ<F>& p, uint32_t k) {
  XYZZ<F> acc = xyzz_zero<F>();
  if (k == 0 || xyzz_is_zero(p)) return acc;
  int top = 31 - __builtin_clz(k);
  acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz_dbl(acc);
    if ((k >> b) & 1) acc = xyzz_add(acc, p);
  }
  return acc;
}

// XYZZ -> affine (identity -> all-zero pair).
template <class F>
ECG_DEV Affine<F> xyzz_to_affine(const XYZZ<F>& p) {
  Affine<F> r;
  if (xyzz_is_zero(p)) {
    r.x = F::zero();
    r.y = F::zero();
    return r;
  }
  F inv = finv(fmul(p.ZZ, p.ZZZ));  // 1/(ZZ*ZZZ)
  F izz = fmul(inv, p.ZZZ);           // 1/ZZ
  F izzz = fmul(inv, p.ZZ);           // 1/ZZZ
  r.x = fmul(p.X, izz);
  r.y = fmul(p.Y, izzz);
  return r;
}

// Jacobian (X, Y, Z) in the reference's G::Curve layout.  Normalised output
// form: (x, y, 1) for a finite point, (0, 1, 0) for the identity (ec.cl:3).
template <class F>
ECG_DEV Jac<F> jac_from_affine_norm(const Affine<F>& a, bool is_identity) {
  Jac<F> r;
  if (is_identity) {
    r.X = F::zero();
    r.Y = F::one();
    r.Z = F::zero();
  } else {
    r.X = a.x;
    r.Y = a.y;
    r.Z = F::one();
  }
  return r;
}

// Jacobian -> XYZZ: ZZ = Z^2, ZZZ = Z^3 (same X, Y).
template <class F>
ECG_DEV XYZZ<F> xyzz_from_jac(const Jac<F>& j) {
  XYZZ<F> r;
  if (fis_zero(j.Z)) return xyzz_zero<F>();
  r.X = j.X;
  r.Y = j.Y;
  r.ZZ = fsqr(j.Z);
  r.ZZZ = fmul(r.ZZ, j.Z);
  return r;
}

template <class F>
ECG_DEV Affine<F> load_affine(const F* xy) {
  Affine<F> a;
  a.x = load(xy);
  a.y = load(xy + 1);
  return a;
}

template <class F>
ECG_DEV void store_xyzz(XYZZ<F>* dst, const XYZZ<F>& p) {
  F* d = reinterpret_cast<F*>(dst);
  store(d + 0, p.X);
  store(d + 1, p.Y);
  store(d + 2, p.ZZ);
  store(d + 3, p.ZZZ);
}

template <class F>
ECG_DEV XYZZ<F> load_xyzz(const XYZZ<F>* src) {
  const F* s = reinterpret_cast<const F*>(src);
  XYZZ<F> p;
  p.X = load(s + 0);
  p.Y = load(s + 1);
  p.ZZ = load(s + 2);
  p.ZZZ = load(s + 3);
  return p;
}

}  // namespace ecg
