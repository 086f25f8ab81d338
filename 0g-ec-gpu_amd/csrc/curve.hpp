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
// Every formula takes an arithmetic policy LZ: false = fully reduced field
// ops (field.hpp strict), true = lazy [0, 2p] representation (field.hpp
// "Lazy"), which the MSM bucket pipeline uses; values are canonicalised
// before they leave the pipeline.
//
// Identity: ZZ == 0 (XYZZ), Z == 0 (Jacobian, as ec.cl's POINT_ZERO=(0,1,0)),
// and the all-zero affine pair (ag-types/src/impls.rs:52-54 GpuRepr).
#pragma once
#include <type_traits>

#include "field.hpp"
#include "field2.hpp"

namespace ecg {

// A curve instance: coordinate field Fq (Fp for G1, Fp2 for G2), scalar field
// Fr, generator constants.  EXT = degree of Fq over the base prime field.
template <class FqP, class FrP, class GenP, int EXT_ = 1>
struct CurveCfg {
  using Fq = std::conditional_t<EXT_ == 1, Fp<FqP>, Fp2<FqP>>;
  using Fr = Fp<FrP>;
  using FqParams = FqP;
  using FrParams = FrP;
  using Gen = GenP;
  static constexpr int EXT = EXT_;
};

using BLS12_381 = CurveCfg<params::bls12_381_fq, params::bls12_381_fr, params::bls12_381_g1>;
using BN254 = CurveCfg<params::bn254_fq, params::bn254_fr, params::bn254_g1>;
// G2 over Fq2 (field2.hpp; ag-build/cl/field2.cl)
using BLS12_381_G2 = CurveCfg<params::bls12_381_fq, params::bls12_381_fr, params::bls12_381_g2, 2>;
using BN254_G2 = CurveCfg<params::bn254_fq, params::bn254_fr, params::bn254_g2, 2>;

// Field element from little-endian u64 words (Montgomery), Fp or Fp2 (c0 first).
template <class P>
ECG_DEV void from_u64_words(Fp<P>& r, const uint64_t* w) {
#pragma unroll
  for (int i = 0; i < Fp<P>::L; i++) r.v[i] = (i & 1) ? (uint32_t)(w[i >> 1] >> 32) : (uint32_t)w[i >> 1];
}
template <class P>
ECG_DEV void from_u64_words(Fp2<P>& r, const uint64_t* w) {
  from_u64_words(r.c0, w);
  from_u64_words(r.c1, w + P::N);
}

// Field-op policy
template <class F, bool LZ>
struct Ops {
  using P = typename F::Params;
  static ECG_DEV F mul(const F& a, const F& b) {
    if constexpr (LZ) return fmul_lz(a, b); else return fmul(a, b);
  }
  static ECG_DEV F sqr(const F& a) {
    if constexpr (LZ) return fsqr_lz(a); else return fsqr(a);
  }
  static ECG_DEV F add(const F& a, const F& b) {
    if constexpr (LZ) return fadd_lz(a, b); else return fadd(a, b);
  }
  static ECG_DEV F sub(const F& a, const F& b) {
    if constexpr (LZ) return fsub_lz(a, b); else return fsub(a, b);
  }
  static ECG_DEV F dbl(const F& a) { return add(a, a); }
  static ECG_DEV F neg(const F& a) {
    if constexpr (LZ) return fneg_lz(a); else return fneg(a);
  }
  static ECG_DEV bool is_zero(const F& a) {
    if constexpr (LZ) return fis_zero_lz(a); else return fis_zero(a);
  }
  static ECG_DEV F canon(const F& a) {
    if constexpr (LZ) return freduce_full(a); else return a;
  }
};

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

template <class F, bool LZ = false>
ECG_DEV bool xyzz_is_zero(const XYZZ<F>& p) {
  return Ops<F, LZ>::is_zero(p.ZZ);
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
template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_dbl_affine(const Affine<F>& a) {
  using O = Ops<F, LZ>;
  F U = O::dbl(a.y);
  F V = O::sqr(U);
  F W = O::mul(U, V);
  F S = O::mul(a.x, V);
  F X2 = O::sqr(a.x);
  F M = O::add(O::dbl(X2), X2);
  XYZZ<F> r;
  r.X = O::sub(O::sub(O::sqr(M), S), S);
  r.Y = O::sub(O::mul(M, O::sub(S, r.X)), O::mul(W, a.y));
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// dbl-2008-s-1 (a = 0): 2 * P
template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_dbl(const XYZZ<F>& p) {
  using O = Ops<F, LZ>;
  if (xyzz_is_zero<F, LZ>(p)) return p;
  F U = O::dbl(p.Y);
  F V = O::sqr(U);
  F W = O::mul(U, V);
  F S = O::mul(p.X, V);
  F X2 = O::sqr(p.X);
  F M = O::add(O::dbl(X2), X2);
  XYZZ<F> r;
  r.X = O::sub(O::sub(O::sqr(M), S), S);
  r.Y = O::sub(O::mul(M, O::sub(S, r.X)), O::mul(W, p.Y));
  r.ZZ = O::mul(V, p.ZZ);
  r.ZZZ = O::mul(W, p.ZZZ);
  return r;
}

// madd-2008-s: P + (x2, y2).  Handles P = O, P = Q (doubling) and P = -Q
// (identity).  `a` must not be the identity (callers skip identity bases).
template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_add_affine(const XYZZ<F>& p, const Affine<F>& a) {
  using O = Ops<F, LZ>;
  if (xyzz_is_zero<F, LZ>(p)) return xyzz_from_affine(a);
  F U2 = O::mul(a.x, p.ZZ);
  F S2 = O::mul(a.y, p.ZZZ);
  F P = O::sub(U2, p.X);
  F R = O::sub(S2, p.Y);
  if (O::is_zero(P)) {
    if (O::is_zero(R)) return xyzz_dbl_affine<F, LZ>(a);
    return xyzz_zero<F>();
  }
  F PP = O::sqr(P);
  F PPP = O::mul(P, PP);
  F Q = O::mul(p.X, PP);
  XYZZ<F> r;
  r.X = O::sub(O::sub(O::sub(O::sqr(R), PPP), Q), Q);
  r.Y = O::sub(O::mul(R, O::sub(Q, r.X)), O::mul(p.Y, PPP));
  r.ZZ = O::mul(p.ZZ, PP);
  r.ZZZ = O::mul(p.ZZZ, PPP);
  return r;
}

// add-2008-s: P + Q, both XYZZ.
template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_add(const XYZZ<F>& p, const XYZZ<F>& q) {
  using O = Ops<F, LZ>;
  if (xyzz_is_zero<F, LZ>(p)) return q;
  if (xyzz_is_zero<F, LZ>(q)) return p;
  F U1 = O::mul(p.X, q.ZZ);
  F U2 = O::mul(q.X, p.ZZ);
  F S1 = O::mul(p.Y, q.ZZZ);
  F S2 = O::mul(q.Y, p.ZZZ);
  F P = O::sub(U2, U1);
  F R = O::sub(S2, S1);
  if (O::is_zero(P)) {
    if (O::is_zero(R)) return xyzz_dbl<F, LZ>(p);
    return xyzz_zero<F>();
  }
  F PP = O::sqr(P);
  F PPP = O::mul(P, PP);
  F Q = O::mul(U1, PP);
  XYZZ<F> r;
  r.X = O::sub(O::sub(O::sub(O::sqr(R), PPP), Q), Q);
  r.Y = O::sub(O::mul(R, O::sub(Q, r.X)), O::mul(S1, PPP));
  r.ZZ = O::mul(O::mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = O::mul(O::mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_neg(const XYZZ<F>& p) {
  XYZZ<F> r = p;
  r.Y = Ops<F, LZ>::neg(p.Y);
  return r;
}

// k * P for a small unsigned scalar (double-and-add from the MSB).
template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_mul_small(const XYZZ<F>& p, uint32_t k) {
  XYZZ<F> acc = xyzz_zero<F>();
  if (k == 0 || xyzz_is_zero<F, LZ>(p)) return acc;
  int top = 31 - __builtin_clz(k);
  acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz_dbl<F, LZ>(acc);
    if ((k >> b) & 1) acc = xyzz_add<F, LZ>(acc, p);
  }
  return acc;
}

// k * P for a canonical multi-word scalar k (8 x u32, little-endian),
// double-and-add from the top set bit.
template <class F, bool LZ = false>
ECG_DEV XYZZ<F> xyzz_mul_scalar(const XYZZ<F>& p, const uint32_t* k) {
  int top = 255;
  while (top >= 0 && !((k[top >> 5] >> (top & 31)) & 1)) top--;
  if (top < 0 || xyzz_is_zero<F, LZ>(p)) return xyzz_zero<F>();
  XYZZ<F> acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz_dbl<F, LZ>(acc);
    if ((k[b >> 5] >> (b & 31)) & 1) acc = xyzz_add<F, LZ>(acc, p);
  }
  return acc;
}

// Canonicalise every coordinate (lazy [0, 2p] -> [0, p)).
template <class F>
ECG_DEV XYZZ<F> xyzz_canon(const XYZZ<F>& p) {
  XYZZ<F> r;
  r.X = freduce_full(p.X);
  r.Y = freduce_full(p.Y);
  r.ZZ = freduce_full(p.ZZ);
  r.ZZZ = freduce_full(p.ZZZ);
  return r;
}

// XYZZ -> affine (identity -> all-zero pair).  Strict inputs.
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
