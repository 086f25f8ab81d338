// Fq2 = Fq[u]/(u^2 + 1) for gfx950: the G2 coordinate field of BLS12-381 and
// BN254.  Replaces ag-build/cl/field2.cl:1-61.  Same representation as
// arkworks' QuadExtField {c0, c1} (two Montgomery Fq elements, c0 first), so
// G2 bases and points cross the C ABI unchanged.
//
// Products use Karatsuba (3 Fq products, field2.cl:34-47), squares the
// complex method (2 products, field2.cl:49-61).  Both exist in the strict
// and the lazy [0, 2p] form (field.hpp), so every curve formula in curve.hpp
// runs over Fp2 through the same Ops<F, LZ> policy.
#pragma once
#include "field.hpp"

namespace ecg {

template <class P>
struct Fp2 {
  using Params = P;
  using Base = Fp<P>;
  static constexpr int L = 2 * Fp<P>::L;  // 32-bit limbs in total
  Fp<P> c0, c1;
  static ECG_DEV Fp2 zero() {
    Fp2 r;
    r.c0 = Fp<P>::zero();
    r.c1 = Fp<P>::zero();
    return r;
  }
  static ECG_DEV Fp2 one() {
    Fp2 r;
    r.c0 = Fp<P>::one();
    r.c1 = Fp<P>::zero();
    return r;
  }
};

template <class P>
ECG_DEV Fp2<P> mk2(const Fp<P>& a, const Fp<P>& b) {
  Fp2<P> r;
  r.c0 = a;
  r.c1 = b;
  return r;
}

// ---- strict (fully reduced) ----
template <class P>
ECG_DEV Fp2<P> fadd(const Fp2<P>& a, const Fp2<P>& b) { return mk2(fadd(a.c0, b.c0), fadd(a.c1, b.c1)); }
template <class P>
ECG_DEV Fp2<P> fsub(const Fp2<P>& a, const Fp2<P>& b) { return mk2(fsub(a.c0, b.c0), fsub(a.c1, b.c1)); }
template <class P>
ECG_DEV Fp2<P> fdbl(const Fp2<P>& a) { return fadd(a, a); }
template <class P>
ECG_DEV Fp2<P> fneg(const Fp2<P>& a) { return mk2(fneg(a.c0), fneg(a.c1)); }
template <class P>
ECG_DEV bool fis_zero(const Fp2<P>& a) { return fis_zero(a.c0) && fis_zero(a.c1); }
template <class P>
ECG_DEV bool feq(const Fp2<P>& a, const Fp2<P>& b) { return feq(a.c0, b.c0) && feq(a.c1, b.c1); }

template <class P>
ECG_DEV Fp2<P> fmul(const Fp2<P>& a, const Fp2<P>& b) {
  const Fp<P> aa = fmul(a.c0, b.c0), bb = fmul(a.c1, b.c1);
  const Fp<P> t = fmul(fadd(a.c0, a.c1), fadd(b.c0, b.c1));
  return mk2(fsub(aa, bb), fsub(fsub(t, aa), bb));
}
template <class P>
ECG_DEV Fp2<P> fsqr(const Fp2<P>& a) {
  const Fp<P> ab = fmul(a.c0, a.c1);
  return mk2(fmul(fadd(a.c0, a.c1), fsub(a.c0, a.c1)), fadd(ab, ab));
}

// 1/(a0 + a1 u) = (a0 - a1 u) / (a0^2 + a1^2)
template <class P>
ECG_DEV Fp2<P> finv(const Fp2<P>& a) {
  const Fp<P> t = finv(fadd(fsqr(a.c0), fsqr(a.c1)));
  return mk2(fmul(a.c0, t), fneg(fmul(a.c1, t)));
}

// ---- lazy [0, 2p] (MSM bucket pipeline) ----
template <class P>
ECG_DEV Fp2<P> fadd_lz(const Fp2<P>& a, const Fp2<P>& b) {
  return mk2(fadd_lz(a.c0, b.c0), fadd_lz(a.c1, b.c1));
}
template <class P>
ECG_DEV Fp2<P> fsub_lz(const Fp2<P>& a, const Fp2<P>& b) {
  return mk2(fsub_lz(a.c0, b.c0), fsub_lz(a.c1, b.c1));
}
template <class P>
ECG_DEV Fp2<P> fneg_lz(const Fp2<P>& a) { return mk2(fneg_lz(a.c0), fneg_lz(a.c1)); }
template <class P>
ECG_DEV bool fis_zero_lz(const Fp2<P>& a) { return fis_zero_lz(a.c0) && fis_zero_lz(a.c1); }
template <class P>
ECG_DEV Fp2<P> freduce_full(const Fp2<P>& a) { return mk2(freduce_full(a.c0), freduce_full(a.c1)); }

template <class P>
ECG_DEV Fp2<P> fmul_lz(const Fp2<P>& a, const Fp2<P>& b) {
  const Fp<P> aa = fmul_lz(a.c0, b.c0), bb = fmul_lz(a.c1, b.c1);
  const Fp<P> t = fmul_lz(fadd_lz(a.c0, a.c1), fadd_lz(b.c0, b.c1));
  return mk2(fsub_lz(aa, bb), fsub_lz(fsub_lz(t, aa), bb));
}
template <class P>
ECG_DEV Fp2<P> fsqr_lz(const Fp2<P>& a) {
  const Fp<P> ab = fmul_lz(a.c0, a.c1);
  return mk2(fmul_lz(fadd_lz(a.c0, a.c1), fsub_lz(a.c0, a.c1)), fadd_lz(ab, ab));
}

// ---- memory ----
template <class P>
ECG_DEV Fp2<P> load(const Fp2<P>* p) {
  const Fp<P>* q = reinterpret_cast<const Fp<P>*>(p);
  return mk2(load(q), load(q + 1));
}
template <class P>
ECG_DEV void store(Fp2<P>* p, const Fp2<P>& a) {
  Fp<P>* q = reinterpret_cast<Fp<P>*>(p);
  store(q, a.c0);
  store(q + 1, a.c1);
}

}  // namespace ecg
