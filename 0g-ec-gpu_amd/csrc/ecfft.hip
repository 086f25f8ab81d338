// FFT over G1 ("EC-FFT", FFTg) for gfx950:  out_k = sum_j omega^(jk) * P_j.
//
// Replaces SingleEcFftKernel::radix_ec_fft (ec-gpu-proxy/src/ec_fft.rs:56-164),
// ag_cuda_ec::ec_fft::radix_ec_fft (ag-cuda-ec/src/ec_fft.rs:12-93) and their
// kernel POINT_radix_fft (ag-build/cl/ec-fft.cl:4-70).  Semantics follow
// serial_ec_fft (ec-gpu-proxy/src/ec_fft_cpu.rs:12-56): natural-order in and
// out, omega a primitive 2^log_n-th root of unity of Fr.
//
// Re-design.  A butterfly here is one full scalar
// multiplication (~255 doublings + ~128 adds, thousands of Fq products) on
// ~200 bytes of point data: the transform is VALU-bound by three orders of
// magnitude over its HBM traffic, so the Stockham/LDS staging that the scalar
// NTT needs buys nothing.  The layout is instead the one that maximises
// independent lanes per launch:
//   1. ecfft_load      Jacobian (any Z) -> XYZZ, written to bit-reversed slots
//   2. ecfft_twiddle   omega^i, i < n/2, canonical (scalar-mul bit source); on
//                      G1 split into GLV halves k = k1 + k2 LAMBDA
//                      (phi(x, y) = (BETA x, y) = LAMBDA P on G1): BLS12-381
//                      by division by its 128-bit LAMBDA, BN254 by the signed
//                      lattice split (254-bit LAMBDA); the twiddle product
//                      becomes two 128-bit products -- half the doublings.
//                      Inputs must be G1 (prime-order subgroup) points, as
//                      ark's G1Projective values are.
//   3. ecfft_stage     log_n launches of n/2 independent radix-2 DIT
//                      butterflies (A, B) -> (A + wB, A - wB), w = 1
//                      butterflies skip the multiply.  G1 points run in the
//                      reduced-radix form of the MSM (curve_rr.hpp: converted
//                      in ecfft_load, back in ecfft_store; ~1.5x faster than
//                      the 32-bit-limb lazy form, which G2 keeps)
//   4. ecfft_store     XYZZ -> normalised Jacobian (x, y, 1) / (0, 1, 0)
#include <atomic>
#include <cstring>
#include <vector>

#ifndef ECG_INST
#error "compile with -DECG_INST=<curve id>"
#endif

#include "ctx.hpp"
#include "curve.hpp"
#include "curve_rr2.hpp"
#include "dispatch.hpp"

namespace ecg {

constexpr int ECFFT_THREADS = 64;


// PF = coordinate field of the butterflies: C::Fq (32-bit limbs, lazy) or the
// reduced-radix FpR / FpR2 of the G1 / G2 base fields (curve_rr*.hpp)
template <class C, class PF>
ECG_DEV XYZZ<PF> to_pf(const XYZZ<typename C::Fq>& p) {
  if constexpr (std::is_same<PF, typename C::Fq>::value) {
    return p;
  } else if constexpr (C::EXT == 2) {
    using Q = typename PF::Params;
    XYZZ<PF> r;
    r.X = rr2_from_std<Q>(p.X);
    r.Y = rr2_from_std<Q>(p.Y);
    r.ZZ = rr2_from_std<Q>(p.ZZ);
    r.ZZZ = rr2_from_std<Q>(p.ZZZ);
    return r;
  } else {
    return pa_from_std_rr<typename PF::Params>(p);
  }
}

template <class C, class PF>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_load_kernel(const typename C::Fq* __restrict__ jac, uint32_t log_n, uint32_t batch,
                      XYZZ<PF>* __restrict__ a) {
  // batch transforms back to back (radix_ec_fft_many runs): point i of the
  // batch is point i mod n of transform i >> log_n
  using F = typename C::Fq;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (batch << log_n)) return;
  Jac<F> j;
  j.X = load(&jac[3 * (size_t)i]);
  j.Y = load(&jac[3 * (size_t)i + 1]);
  j.Z = load(&jac[3 * (size_t)i + 2]);
  const uint32_t il = i & ((1u << log_n) - 1);
  const uint32_t r = log_n ? (__brev(il) >> (32 - log_n)) : 0u;
  store_xyzz(&a[(i - il) + r], to_pf<C, PF>(xyzz_from_jac(j)));
}

template <class C>
constexpr bool has_glv() {
  return C::EXT == 1 && C::Gen::GLV != 0;
}

// GLV split of a canonical scalar k < r (BLS12-381 G1): k = k2 * LAMBDA + k1,
// 0 <= k1 < LAMBDA < 2^128, k2 < r / LAMBDA < 2^128 (bit-serial division by
// the fixed 128-bit LAMBDA; runs once per twiddle when the table is built).
template <class C>
ECG_DEV void glv_split(const uint32_t* k, uint32_t* k1, uint32_t* k2) {
  uint32_t lam[5];
#pragma unroll
  for (int i = 0; i < 4; i++) lam[i] = (i & 1) ? (uint32_t)(C::Gen::LAMBDA[i >> 1] >> 32) : (uint32_t)C::Gen::LAMBDA[i >> 1];
  lam[4] = 0;
  uint32_t rem[5] = {0, 0, 0, 0, 0};
  uint32_t q[4] = {0, 0, 0, 0};
  for (int b = 255; b >= 0; b--) {
#pragma unroll
    for (int i = 4; i > 0; i--) rem[i] = (rem[i] << 1) | (rem[i - 1] >> 31);
    rem[0] = (rem[0] << 1) | ((k[b >> 5] >> (b & 31)) & 1);
    bool ge = true;  // rem >= lam ?
#pragma unroll
    for (int i = 4; i >= 0; i--) {
      if (rem[i] != lam[i]) {
        ge = rem[i] > lam[i];
        break;
      }
    }
    if (ge) {
      uint32_t br = 0;
#pragma unroll
      for (int i = 0; i < 5; i++) {
        const uint64_t d = (uint64_t)rem[i] - lam[i] - br;
        rem[i] = (uint32_t)d;
        br = (uint32_t)(d >> 63);
      }
      if (b < 128) q[b >> 5] |= 1u << (b & 31);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    k1[i] = rem[i];
    k2[i] = q[i];
  }
}

// 32-bit words of a u64 constant array
template <int N>
ECG_DEV void words_of(const uint64_t (&v)[N], uint32_t* w) {
#pragma unroll
  for (int i = 0; i < N; i++) {
    w[2 * i] = (uint32_t)v[i];
    w[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
}

// c = floor((k g + 2^319) / 2^320) for k < 2^256 (8 words) and g < 2^256 (8
// words): the rounded k * (b / r) of the lattice split, c < 2^128
ECG_DEV void glv_round(const uint32_t* k, const uint32_t* g, uint32_t* c) {
  uint32_t pr[16];
#pragma unroll
  for (int i = 0; i < 16; i++) pr[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)k[i] * g[j] + pr[i + j] + carry;
      pr[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    pr[i + 8] = (uint32_t)carry;
  }
  uint64_t t = (uint64_t)pr[9] + 0x80000000u;  // + 2^319
  pr[9] = (uint32_t)t;
#pragma unroll
  for (int i = 10; i < 14; i++) {
    t = (uint64_t)pr[i] + (t >> 32);
    c[i - 10] = (uint32_t)t;
  }
}

// low 128 bits of x * y (4 words each)
ECG_DEV void mul_lo128(const uint32_t* x, const uint32_t* y, uint32_t* z) {
  uint32_t r[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; i + j < 4; j++) {
      const uint64_t t = (uint64_t)x[i] * y[j] + r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) z[i] = r[i];
}

ECG_DEV void sub128(uint32_t* x, const uint32_t* y) {  // x -= y mod 2^128
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t d = (uint64_t)x[i] - y[i] - br;
    x[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
}

// |v| with the sign in bit 127 (|v| < 2^126: GLV_LATTICE bound)
ECG_DEV void sign_magnitude128(uint32_t* v) {
  if (!(v[3] >> 31)) return;
  const uint32_t z[4] = {0, 0, 0, 0};
  uint32_t m[4] = {z[0], z[1], z[2], z[3]};
  sub128(m, v);
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = m[i];
  v[3] |= 0x80000000u;
}

// GLV lattice split of k < r (BN254 G1, GLV = 2; constants and bounds in
// tools/gen_params.py): k = k1 + k2 LAMBDA mod r, each half as a 127-bit
// magnitude with its sign in bit 127.  Once per twiddle, when the table is
// built.
template <class C>
ECG_DEV void glv_lattice_split(const uint32_t* k, uint32_t* k1, uint32_t* k2) {
  using G = typename C::Gen;
  uint32_t g1[8], g2[8], a1[4], a2[4], nb1[4], b2[4], c1[4], c2[4], t[4];
  words_of(G::G1, g1);
  words_of(G::G2, g2);
  words_of(G::A1, a1);
  words_of(G::A2, a2);
  words_of(G::NB1, nb1);
  words_of(G::B2, b2);
  glv_round(k, g1, c1);
  glv_round(k, g2, c2);
#pragma unroll
  for (int i = 0; i < 4; i++) k1[i] = k[i];
  mul_lo128(c1, a1, t);
  sub128(k1, t);
  mul_lo128(c2, a2, t);
  sub128(k1, t);
  mul_lo128(c1, nb1, k2);
  mul_lo128(c2, b2, t);
  sub128(k2, t);
  sign_magnitude128(k1);
  sign_magnitude128(k2);
}

// the sign bit of a lattice half (GLV = 2), cleared from k; false otherwise
template <class C>
ECG_DEV bool glv_take_sign(uint32_t* k) {
  if constexpr (C::Gen::GLV == 2) {
    const bool neg = k[3] >> 31;
    k[3] &= 0x7fffffffu;
    return neg;
  } else {
    return false;
  }
}

// Twiddle table entry i (2 x uint4): canonical omega^i, or its GLV halves
// (k1 | k2) for curves with the endomorphism (BLS12-381: by division by the
// 128-bit LAMBDA; BN254: the lattice split, signed).
template <class C>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_twiddle_kernel(Fp<typename C::FrParams> omega, uint32_t half, uint4* __restrict__ tw) {
  using S = Fp<typename C::FrParams>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  S w = from_mont(fpow_u32(omega, i));
  if constexpr (has_glv<C>()) {
    uint32_t k1[4], k2[4];
    if constexpr (C::Gen::GLV == 2)
      glv_lattice_split<C>(w.v, k1, k2);
    else
      glv_split<C>(w.v, k1, k2);
    tw[2 * i] = make_uint4(k1[0], k1[1], k1[2], k1[3]);
    tw[2 * i + 1] = make_uint4(k2[0], k2[1], k2[2], k2[3]);
  } else {
    tw[2 * i] = make_uint4(w.v[0], w.v[1], w.v[2], w.v[3]);
    tw[2 * i + 1] = make_uint4(w.v[4], w.v[5], w.v[6], w.v[7]);
  }
}

// k1 P + k2 phi(P) by a joint (Straus-Shamir) double-and-add over the 128-bit
// halves: one doubling per bit of the longer half and one full add from the
// table {P, phi P, P + phi P} per nonzero bit pair.  The table lives in a
// per-butterfly global slot (L2-resident), keeping VGPRs for the chain.
template <class C, class PF>
ECG_DEV XYZZ<PF> glv_joint_mul(const XYZZ<PF>& P0, const uint32_t* k1s, const uint32_t* k2s, XYZZ<PF>* tab) {
  using F = typename C::Fq;
  if (pa_is_zero(P0)) return P0;
  uint32_t k1[4] = {k1s[0], k1s[1], k1s[2], k1s[3]}, k2[4] = {k2s[0], k2s[1], k2s[2], k2s[3]};
  const bool n1 = glv_take_sign<C>(k1), n2 = glv_take_sign<C>(k2);  // lattice halves are signed
  F beta;
  from_u64_words(beta, C::Gen::BETA);
  const XYZZ<PF> P = n1 ? pa_neg(P0) : P0;
  XYZZ<PF> phi = n2 ? pa_neg(P0) : P0;
  phi.X = pa_mul_const(P0.X, beta);
  store_xyzz(&tab[0], P);
  store_xyzz(&tab[1], phi);
  store_xyzz(&tab[2], pa_add(P, phi));
  int top = 127;
  while (top >= 0 && !(((k1[top >> 5] | k2[top >> 5]) >> (top & 31)) & 1)) top--;
  if (top < 0) return xyzz_zero<PF>();
  const uint32_t d0 = ((k1[top >> 5] >> (top & 31)) & 1) | (((k2[top >> 5] >> (top & 31)) & 1) << 1);
  XYZZ<PF> acc = load_xyzz(&tab[d0 - 1]);
  for (int b = top - 1; b >= 0; b--) {
    acc = pa_dbl(acc);
    const uint32_t d = ((k1[b >> 5] >> (b & 31)) & 1) | (((k2[b >> 5] >> (b & 31)) & 1) << 1);
    if (d) acc = pa_add(acc, load_xyzz(&tab[d - 1]));
  }
  return acc;
}

// Stage s of the DIT: half-size h = 2^s; butterfly t pairs i0 = (t >> s) *
// 2h + j and i1 = i0 + h, j = t mod h, twiddle omega^(j * n / 2h)
// (serial_ec_fft's w = w_m^j, ec_fft_cpu.rs:35-49).
template <class C, class PF>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_stage_kernel(XYZZ<PF>* __restrict__ a, const uint4* __restrict__ tw, uint32_t log_n, uint32_t s,
                       XYZZ<PF>* __restrict__ glv_tab) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (1u << (log_n - 1))) return;
  const uint32_t h = 1u << s;
  const uint32_t j = t & (h - 1);
  const uint32_t i0 = ((t >> s) << (s + 1)) + j, i1 = i0 + h;
  XYZZ<PF> A = load_xyzz(&a[i0]);
  XYZZ<PF> B = load_xyzz(&a[i1]);
  if (j != 0) {
    const uint32_t e = j << (log_n - 1 - s);
    const uint4 lo = tw[2 * e], hi = tw[2 * e + 1];
    if constexpr (has_glv<C>()) {
      const uint32_t k1[4] = {lo.x, lo.y, lo.z, lo.w}, k2[4] = {hi.x, hi.y, hi.z, hi.w};
      B = glv_joint_mul<C, PF>(B, k1, k2, glv_tab + 3 * (size_t)t);
    } else {
      const uint32_t k[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      B = pa_mul_scalar(B, k);
    }
  }
  store_xyzz(&a[i0], pa_add(A, B));
  store_xyzz(&a[i1], pa_add(A, pa_neg(B)));
}

// ---------------------------------------------------------------------------
// Windowed stage (default): the butterflies of the small transforms 0g runs
// (2^10..2^16 points: 512..32768 butterflies, under one wave per SIMD) are
// latency-bound -- a stage takes one scalar multiplication's dependency chain,
// whatever the lane count -- so the stage shortens the chain:
//  * signed 4-bit windows with no carry pass: K = k + sum_i 8 * 16^i, digit i
//    = nibble i of K minus 8, in [-8, 7]; a table m P (m = 1..8, 4 levels of
//    adds/doublings) in the lane's global slot; per digit 4 doublings and one
//    add (15/16 of digits are nonzero): 128 doublings + 32 adds per 128 bits
//    instead of the bit ladder's 128 + 64 (+ 96 for the joint GLV ladder);
//  * on GLV curves two lanes per butterfly, one per half (k1 P and k2 phi(P)),
//    joined by a lane shuffle and one add: the joint ladder's 128 doublings
//    + ~96 adds become 128 doublings + ~34 adds on the critical path.
// ---------------------------------------------------------------------------
constexpr int ECFFT_TAB = 8;  // table entries per lane (m P, m = 1..8)

// r.Y = -r.Y where c, word by word (no whole-struct copy under a condition)
template <class PF>
ECG_DEV XYZZ<PF> neg_if(const XYZZ<PF>& p, bool c) {
  const XYZZ<PF> n = pa_neg(p);
  constexpr int NW = (int)(sizeof(PF) / 4);
  uint32_t w[NW], nw[NW];
  __builtin_memcpy(w, &p.Y, sizeof(PF));
  __builtin_memcpy(nw, &n.Y, sizeof(PF));
#pragma unroll
  for (int i = 0; i < NW; i++) w[i] = c ? nw[i] : w[i];
  XYZZ<PF> r = p;
  __builtin_memcpy(&r.Y, w, sizeof(PF));
  return r;
}

template <class T>
ECG_DEV T sel_words(bool c, const T& a, const T& b) {  // c ? a : b
  constexpr int NW = (int)(sizeof(T) / 4);
  uint32_t wa[NW], wb[NW];
  __builtin_memcpy(wa, &a, sizeof(T));
  __builtin_memcpy(wb, &b, sizeof(T));
#pragma unroll
  for (int i = 0; i < NW; i++) wb[i] = c ? wa[i] : wb[i];
  T r;
  __builtin_memcpy(&r, wb, sizeof(T));
  return r;
}

template <int X = 1, class T>
ECG_DEV T shfl_xor1(const T& v) {  // the partner lane's value (lanes u <-> u ^ X)
  constexpr int NW = (int)(sizeof(T) / 4);
  uint32_t w[NW];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int i = 0; i < NW; i++) w[i] = (uint32_t)__shfl_xor((int)w[i], X);
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}

// k P, k little-endian in W words (signed 4-bit windows, see above)
template <int W, int PM = 0, class PF>
ECG_DEV XYZZ<PF> win_mul(const XYZZ<PF>& P, const uint32_t* k, XYZZ<PF>* __restrict__ tab) {
  uint32_t K[W + 1];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < W; i++) {
    c += (uint64_t)k[i] + 0x88888888u;
    K[i] = (uint32_t)c;
    c >>= 32;
  }
  K[W] = (uint32_t)c + 8u;  // digit 8W in {0, 1}
  // table m P, m = 1..8: four levels (2P; 3P, 4P; 5P, 6P, 8P; 7P)
  store_xyzz(&tab[0], P);
  const XYZZ<PF> P2 = pp_dbl<PM>(P);
  store_xyzz(&tab[1], P2);
  const XYZZ<PF> P3 = pp_add<PM>(P2, P);
  store_xyzz(&tab[2], P3);
  const XYZZ<PF> P4 = pp_dbl<PM>(P2);
  store_xyzz(&tab[3], P4);
  store_xyzz(&tab[4], pp_add<PM>(P4, P));
  const XYZZ<PF> P6 = pp_dbl<PM>(P3);
  store_xyzz(&tab[5], P6);
  store_xyzz(&tab[6], pp_add<PM>(P6, P));
  store_xyzz(&tab[7], pp_dbl<PM>(P4));
  XYZZ<PF> acc = xyzz_zero<PF>();
#pragma unroll 1
  for (int i = 8 * W; i >= 0; i--) {
    uint32_t word = K[0];
#pragma unroll
    for (int q = 1; q <= W; q++) word = (i >> 3) == q ? K[q] : word;
    const int d = (int)((word >> ((i & 7) * 4)) & 15u) - 8;
    const XYZZ<PF> T = load_xyzz(&tab[d < 0 ? -d - 1 : d > 0 ? d - 1 : 0]);  // issued before the doublings
#pragma unroll 1
    for (int b = 0; b < 4; b++) acc = pp_dbl<PM>(acc);
    if (d != 0) acc = pp_add<PM>(acc, neg_if(T, d < 0));
  }
  return acc;
}

// Stage s (as ecfft_stage_kernel) with windowed products; GLV curves: lanes
// 2u, 2u + 1 share butterfly u (half 0: k1 P, half 1: k2 phi(P)).  With PM = 1
// every lane of that layout becomes a lane pair (lanes 2v, 2v + 1), with PM = 4
// a quad (lanes 4v .. 4v + 3), sharing each point operation's products
// (pp_dbl / pp_add); the GLV partner is then lane ^ 2 or lane ^ 4.
template <class C, class PF, int PM>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_stage_win_kernel(XYZZ<PF>* __restrict__ a, const uint4* __restrict__ tw, uint32_t log_n, uint32_t s,
                           uint32_t batch, XYZZ<PF>* __restrict__ tabs) {
  constexpr bool glv = has_glv<C>();
  constexpr uint32_t PB = pp_lanes_log<PM>();  // log2 lanes per point operation
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lanes_log = (glv ? log_n : log_n - 1) + PB;  // lanes per transform
  if (g >= (batch << lanes_log)) return;               // the lanes of a butterfly leave together
  a += (size_t)(g >> lanes_log) << log_n;              // transform g >> lanes_log of the batch
  const uint32_t gl = (g & ((1u << lanes_log) - 1)) >> PB;
  const uint32_t role = g & ((1u << PB) - 1);           // lane within the point operation
  const bool lead = role == 0;                          // the lane that stores
  const uint32_t t = glv ? gl >> 1 : gl;
  const uint32_t half = glv ? (gl & 1) : 0u;
  const uint32_t h = 1u << s;
  const uint32_t j = t & (h - 1);
  const uint32_t i0 = ((t >> s) << (s + 1)) + j, i1 = i0 + h;
  const XYZZ<PF> A = load_xyzz(&a[i0]);
  const XYZZ<PF> B = load_xyzz(&a[i1]);
  XYZZ<PF> R = B;
  if (j != 0) {  // uniform within a pair
    const uint32_t e = j << (log_n - 1 - s);
    if constexpr (glv) {
      const uint4 kk = tw[2 * e + half];
      uint32_t k[4] = {kk.x, kk.y, kk.z, kk.w};
      const bool kneg = glv_take_sign<C>(k);  // BN254: signed lattice halves (uniform per half)
      typename C::Fq beta;
      from_u64_words(beta, C::Gen::BETA);
      XYZZ<PF> Bh = neg_if(B, kneg);
      Bh.X = sel_words(half != 0, pa_mul_const(B.X, beta), B.X);  // phi(x, y) = (beta x, y)
      const XYZZ<PF> Rh = win_mul<4, PM>(Bh, k, tabs + (size_t)ECFFT_TAB * g);
      R = pp_add<PM>(Rh, shfl_xor1<1 << PB>(Rh));
    } else {
      const uint4 lo = tw[2 * e], hi = tw[2 * e + 1];
      const uint32_t k[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      R = win_mul<8, PM>(B, k, tabs + (size_t)ECFFT_TAB * g);
    }
  }
  if constexpr (glv) {  // half 0 writes A + wB, half 1 A - wB
    const XYZZ<PF> o = pp_add<PM>(A, neg_if(R, half != 0));
    if (lead) store_xyzz(&a[half ? i1 : i0], o);
  } else if constexpr (PM != 0) {  // lanes 0 and 1 of the operation store one output each
    const XYZZ<PF> o0 = pp_add<PM>(A, R);
    const XYZZ<PF> o1 = pp_add<PM>(A, pa_neg(R));
    if (role < 2) store_xyzz(&a[lead ? i0 : i1], lead ? o0 : o1);
  } else {
    store_xyzz(&a[i0], pa_add(A, R));
    store_xyzz(&a[i1], pa_add(A, pa_neg(R)));
  }
}

// ---------------------------------------------------------------------------
// Radix-2^d stages (the small transforms, where a stage's cost is its one
// scalar multiplication's chain, not its work).  One radix-2^d DIT stage does
// the work of d radix-2 stages with ONE multiplication on its critical path:
// over bit-reversed input, block blk of M = 2^(s+d) points holds R = 2^d
// transformed sub-blocks of 2^s points -- sub-block m transforms the inputs
// congruent to m' = brev_d(m) mod R -- and output j + q 2^s (j < 2^s, q < R)
// of the block is
//     sum_{m < R} omega^E(j, m, q) in[blk M + j + m 2^s],
//     E = (n/M) ((j + q 2^s) m' mod M) = (n/M) j m' + q m' (n/R)  (mod n).
// E(q + R/2) = E(q) + m' n/2: for odd m' the product is negated, for even m'
// it is the same, so a stage needs n (R - 1) / 2 distinct products (R = 2: the
// radix-2 butterfly's n/2).  Kernel 1 computes them (windowed, GLV halves,
// lane pairs / quads as the radix-2 stage); kernel 2 sums each output's R
// terms (its m = 0 term is the input itself) into the other point buffer.
// The work grows as 2 (R - 1) / d over radix-2 stages, the chain shrinks d
// times; ecfft_radix_plan picks d per size.
// ---------------------------------------------------------------------------
struct RadixStage {
  uint32_t log_n, s, d;
  uint32_t np;     // distinct products per transform: (n / 2) (R - 1)
  uint32_t batch;
};

template <class C, class PF, int PM>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_rprod_kernel(const XYZZ<PF>* __restrict__ a, XYZZ<PF>* __restrict__ prod, const uint4* __restrict__ tw,
                       RadixStage st, XYZZ<PF>* __restrict__ tabs) {
  constexpr bool glv = has_glv<C>();
  constexpr uint32_t PB = pp_lanes_log<PM>();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t per_op = (glv ? 2u : 1u) << PB;  // lanes per product
  if (g >= st.batch * st.np * per_op) return;      // the lanes of a product leave together
  const uint32_t role = g & ((1u << PB) - 1);
  uint32_t op = g >> PB;
  const uint32_t half = glv ? (op & 1u) : 0u;
  if (glv) op >>= 1;
  const uint32_t tr = op / st.np, t = op - tr * st.np;
  const uint32_t d = st.d, s = st.s, R1 = (1u << d) - 1;
  const uint32_t q = t & ((1u << (d - 1)) - 1);
  const uint32_t u = t >> (d - 1);
  const uint32_t j = u & ((1u << s) - 1);
  const uint32_t v = u >> s;
  const uint32_t blk = v / R1, m = v - blk * R1 + 1;
  const uint32_t n = 1u << st.log_n, half_n = n >> 1;
  const uint32_t mr = __brev(m) >> (32 - d);  // sub-block m holds the inputs = brev_d(m) mod R
  const uint32_t E = (((j * mr) << (st.log_n - s - d)) + ((q * mr) << (st.log_n - d))) & (n - 1);
  const uint32_t e = E & (half_n - 1);
  const XYZZ<PF> B = load_xyzz(&a[(size_t)tr * n + (blk << (s + d)) + j + (m << s)]);
  XYZZ<PF> P = B;
  if (e != 0) {  // uniform within a product's lanes
    if constexpr (glv) {
      const uint4 kk = tw[2 * e + half];
      uint32_t k[4] = {kk.x, kk.y, kk.z, kk.w};
      const bool kneg = glv_take_sign<C>(k);
      typename C::Fq beta;
      from_u64_words(beta, C::Gen::BETA);
      XYZZ<PF> Bh = neg_if(B, kneg);
      Bh.X = sel_words(half != 0, pa_mul_const(B.X, beta), B.X);
      const XYZZ<PF> Rh = win_mul<4, PM>(Bh, k, tabs + (size_t)ECFFT_TAB * g);
      P = pp_add<PM>(Rh, shfl_xor1<1 << PB>(Rh));
    } else {
      const uint4 lo = tw[2 * e], hi = tw[2 * e + 1];
      const uint32_t k[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      P = win_mul<8, PM>(B, k, tabs + (size_t)ECFFT_TAB * g);
    }
  }
  if (role == 0 && half == 0) store_xyzz(&prod[(size_t)tr * st.np + t], neg_if(P, E >= half_n));
}

template <class C, class PF, int PM>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_rsum_kernel(const XYZZ<PF>* __restrict__ a, const XYZZ<PF>* __restrict__ prod, XYZZ<PF>* __restrict__ out,
                      RadixStage st) {
  constexpr uint32_t PB = pp_lanes_log<PM>();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (st.batch << (st.log_n + PB))) return;
  const uint32_t op = g >> PB;
  const uint32_t tr = op >> st.log_n, o = op & ((1u << st.log_n) - 1);
  const uint32_t d = st.d, s = st.s, R1 = (1u << d) - 1;
  const uint32_t blk = o >> (s + d), oi = o & ((1u << (s + d)) - 1);
  const uint32_t j = oi & ((1u << s) - 1), q = oi >> s;
  const uint32_t qh = q & ((1u << (d - 1)) - 1);
  const bool upper = q >> (d - 1);
  const XYZZ<PF>* pr = prod + (size_t)tr * st.np + ((((size_t)blk * R1) << s) << (d - 1));
  XYZZ<PF> acc = load_xyzz(&a[((size_t)tr << st.log_n) + (blk << (s + d)) + j]);
  XYZZ<PF> nxt = load_xyzz(&pr[((size_t)j << (d - 1)) + qh]);
#pragma unroll 1
  for (uint32_t m = 1; m <= R1; m++) {
    const XYZZ<PF> cur = nxt;
    if (m < R1) nxt = load_xyzz(&pr[((((size_t)m << s) + j) << (d - 1)) + qh]);  // one ahead
    acc = pp_add<PM>(acc, neg_if(cur, upper && ((m >> (d - 1)) & 1)));  // odd brev_d(m)
  }
  if ((g & ((1u << PB) - 1)) == 0) store_xyzz(&out[((size_t)tr << st.log_n) + o], acc);
}

static uint32_t ecfft_pairs_max() {  // A/B: ECG_ECFFT_PAIRS = 0 / 1 (single lanes), 2 (pairs), 4 (quads)
  static const uint32_t v = [] {
    const char* e = getenv("ECG_ECFFT_PAIRS");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 4u;
  }();
  return v;
}

// Log-radices of the stages of a 2^log_n transform (batch of `batch`): stages
// of at most dmax radix-2 rounds each, balanced.  dmax = 1 is the radix-2
// chain.  A/B: ECG_ECFFT_RADIX pins dmax (1 = radix-2 stages only).
// ecg_ec_fft_set_radix (process-wide A/B and test knob; 0 = automatic)
extern std::atomic<int> ecfft_radix_pin;
#if ECG_INST == 0
std::atomic<int> ecfft_radix_pin{0};
#endif

static uint32_t ecfft_radix_max(uint32_t log_n, uint32_t batch) {
  const int api = ecfft_radix_pin.load(std::memory_order_relaxed);
  if (api > 0) return (uint32_t)api;
  static const int pinned = [] {
    const char* e = getenv("ECG_ECFFT_RADIX");
    const long v = e ? strtol(e, nullptr, 10) : 0;
    return v >= 1 && v <= 8 ? (int)v : 0;
  }();
  if (pinned) return (uint32_t)pinned;
  // by the points of the whole launch (batch x n): below ~2^15 points a stage
  // costs its chain, so fewer, wider stages win until their (R - 1) / (d / 2)
  // times larger product count fills the chip.  Measured on both G1 curves
  // (profiles/r05/ecfft_radix_sweep.log): 2^6 2.2x, 2^10 2.5x, 2^12 2.0x,
  // 2^14 1.15x over radix-2 stages; 2^15 up and 32 x 2^10 keep radix-2.
  uint32_t lt = log_n;
  for (uint32_t b = batch; b > 1; b >>= 1) lt++;
  const uint32_t d = lt <= 7 ? log_n : lt == 8 ? 4u : lt <= 10 ? 5u : lt == 11 ? 4u : lt == 12 ? 3u : lt <= 14 ? 2u : 1u;
  return d < log_n ? d : log_n;
}

static std::vector<uint32_t> ecfft_radix_plan(uint32_t log_n, uint32_t dmax) {
  std::vector<uint32_t> plan;
  if (log_n == 0) return plan;
  const uint32_t nst = (log_n + dmax - 1) / dmax;
  for (uint32_t k = 0; k < nst; k++) plan.push_back(log_n / nst + (k < log_n % nst ? 1u : 0u));
  return plan;
}

static bool ecfft_win_enabled() {  // A/B switch: ECG_ECFFT_WIN=0 keeps the bit ladders (ecfft_stage_kernel)
  static const bool v = [] {
    const char* e = getenv("ECG_ECFFT_WIN");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <class C, class PF>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_store_kernel(const XYZZ<PF>* __restrict__ a, uint32_t n, typename C::Fq* __restrict__ jac) {
  using F = typename C::Fq;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  XYZZ<F> p = xyzz_canon(pa_to_std(load_xyzz(&a[i])));
  const bool id = xyzz_is_zero(p);
  Jac<F> j = jac_from_affine_norm(xyzz_to_affine(p), id);
  store(&jac[3 * (size_t)i], j.X);
  store(&jac[3 * (size_t)i + 1], j.Y);
  store(&jac[3 * (size_t)i + 2], j.Z);
}

static inline uint32_t ecfft_blocks(size_t n) { return (uint32_t)((n + ECFFT_THREADS - 1) / ECFFT_THREADS); }

static bool ecfft_rr_enabled() {  // A/B switch: ECG_ECFFT_RR=0 keeps the 32-bit-limb butterflies
  static const bool v = [] {
    const char* e = getenv("ECG_ECFFT_RR");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <class C, class PF>
static int ecfft_pf(ecg_ctx* ctx, void* d_jac, const uint64_t* omega, uint32_t log_n, hipStream_t s,
                    ecg_abort_cb abort_cb, void* user, uint32_t batch) {
  using F = typename C::Fq;
  using S = Fp<typename C::FrParams>;
  const uint32_t n = 1u << log_n;
  // windowed stages for the reduced-radix point forms (the 32-bit-limb forms
  // are the A/B baseline and keep the bit ladders)
  const bool win = !std::is_same<PF, F>::value && ecfft_win_enabled();
  if (batch > 1 && (!win || log_n == 0)) {  // batched stages are a windowed-form feature
    for (uint32_t b = 0; b < batch; b++)
      ECG_TRY((ecfft_pf<C, PF>(ctx, (F*)d_jac + 3 * (size_t)b * n, omega, log_n, s, abort_cb, user, 1)));
    return ECG_OK;
  }
  const size_t nb = (size_t)batch * n;
  void *a, *tw, *gt = nullptr;
  ECG_TRY(ws_get(ctx, "ecfft_pts", nb * sizeof(XYZZ<PF>), &a));
  ECG_TRY(ws_get(ctx, "ecfft_tw", (size_t)(n / 2 + 1) * 32, &tw));
  // lane pairs / quads while the widened stage still leaves each SIMD at most
  // one wave (2^16 lanes): pairs made 2^10-2^14 G1 stages 33 % faster, but at
  // 2^16 (one wave per SIMD unpaired) they are 26 % slower
  // (profiles/r04/lane_pairs_ab.txt).  ECG_ECFFT_PAIRS: 0 single lanes,
  // 2 pairs at most, 4 (default) quads where they fit.
  const size_t lanes1 = has_glv<C>() && win ? nb : (size_t)batch * (n / 2);
  const uint32_t pmax = win && PairOps<PF>::ok ? ecfft_pairs_max() : 1u;
  const uint32_t widen = QuadOps<PF>::ok && pmax >= 4 && lanes1 <= ((size_t)1 << 14)  ? 4u
                         : pmax >= 2 && lanes1 <= ((size_t)1 << 15)                 ? 2u
                                                                                    : 1u;
  const bool pairs = widen > 1;
  // stage lanes: 2 per butterfly on GLV curves, times the lanes per operation
  const size_t lanes = lanes1 * widen + 1;
  if (win)
    ECG_TRY(ws_get(ctx, "ecfft_tab", lanes * ECFFT_TAB * sizeof(XYZZ<PF>), &gt));
  else if (has_glv<C>())
    ECG_TRY(ws_get(ctx, "ecfft_glv", (size_t)(n / 2 + 1) * 3 * sizeof(XYZZ<PF>), &gt));
  S om;
  memcpy(om.v, omega, sizeof(om.v));
  hipLaunchKernelGGL((ecfft_load_kernel<C, PF>), dim3(ecfft_blocks(nb)), dim3(ECFFT_THREADS), 0, s, (const F*)d_jac,
                     log_n, batch, (XYZZ<PF>*)a);
  ECG_HIP(hipGetLastError());
  if (log_n > 0) {
    hipLaunchKernelGGL(ecfft_twiddle_kernel<C>, dim3(ecfft_blocks(n / 2)), dim3(ECFFT_THREADS), 0, s, om, n / 2,
                       (uint4*)tw);
    ECG_HIP(hipGetLastError());
  }
  kt_reset(ctx, "ecfft_stage");
  // radix-2^d stages (see ecfft_rprod_kernel) for the latency-bound sizes
  if constexpr (!std::is_same<PF, F>::value) {
    const std::vector<uint32_t> plan = win ? ecfft_radix_plan(log_n, ecfft_radix_max(log_n, batch))
                                           : std::vector<uint32_t>{};
    bool radix = false;
    for (uint32_t d : plan) radix = radix || d > 1;
    if (radix) {
      const size_t half_lanes = has_glv<C>() ? 2 : 1;
      size_t np_max = 0;
      for (uint32_t d : plan) np_max = std::max(np_max, (size_t)(n / 2) * ((1u << d) - 1));
      auto widen_for = [&](size_t lanes1) -> uint32_t {
        return QuadOps<PF>::ok && pmax >= 4 && lanes1 <= ((size_t)1 << 14)  ? 4u
               : PairOps<PF>::ok && pmax >= 2 && lanes1 <= ((size_t)1 << 15) ? 2u
                                                                            : 1u;
      };
      void *a2, *prod, *tabs;
      ECG_TRY(ws_get(ctx, "ecfft_pts2", nb * sizeof(XYZZ<PF>), &a2));
      ECG_TRY(ws_get(ctx, "ecfft_prod", (size_t)batch * np_max * sizeof(XYZZ<PF>), &prod));
      size_t tab_lanes = 0;  // the widest product launch of the plan
      for (uint32_t d : plan) {
        const size_t pl1 = (size_t)batch * (n / 2) * ((1u << d) - 1) * half_lanes;
        tab_lanes = std::max(tab_lanes, pl1 * widen_for(pl1));
      }
      ECG_TRY(ws_get(ctx, "ecfft_rtab", (tab_lanes + 1) * ECFFT_TAB * sizeof(XYZZ<PF>), &tabs));
      XYZZ<PF>* cur = (XYZZ<PF>*)a;
      XYZZ<PF>* oth = (XYZZ<PF>*)a2;
      uint32_t s0 = 0;
      for (uint32_t d : plan) {
        if (abort_cb && abort_cb(user)) {  // ec_fft.rs:112-116, once per round
          (void)hipStreamSynchronize(s);
          return ECG_ABORTED;
        }
        const RadixStage rs{log_n, s0, d, (n / 2) * ((1u << d) - 1), batch};
        ECG_TRY(kt_begin(ctx, "ecfft_stage", s));
        const size_t pl1 = (size_t)batch * rs.np * half_lanes;
        const uint32_t wp = widen_for(pl1);
        const size_t plan_lanes = pl1 * wp;
        if (wp == 4) {
          if constexpr (QuadOps<PF>::ok)
            hipLaunchKernelGGL((ecfft_rprod_kernel<C, PF, 4>), dim3(ecfft_blocks(plan_lanes)), dim3(ECFFT_THREADS), 0,
                               s, cur, (XYZZ<PF>*)prod, (const uint4*)tw, rs, (XYZZ<PF>*)tabs);
        } else if (wp == 2) {
          if constexpr (PairOps<PF>::ok)
            hipLaunchKernelGGL((ecfft_rprod_kernel<C, PF, 1>), dim3(ecfft_blocks(plan_lanes)), dim3(ECFFT_THREADS), 0,
                               s, cur, (XYZZ<PF>*)prod, (const uint4*)tw, rs, (XYZZ<PF>*)tabs);
        } else {
          hipLaunchKernelGGL((ecfft_rprod_kernel<C, PF, 0>), dim3(ecfft_blocks(plan_lanes)), dim3(ECFFT_THREADS), 0, s,
                             cur, (XYZZ<PF>*)prod, (const uint4*)tw, rs, (XYZZ<PF>*)tabs);
        }
        ECG_HIP(hipGetLastError());
        const uint32_t ws = widen_for(nb);
        if (ws == 4) {
          if constexpr (QuadOps<PF>::ok)
            hipLaunchKernelGGL((ecfft_rsum_kernel<C, PF, 4>), dim3(ecfft_blocks(nb * 4)), dim3(ECFFT_THREADS), 0, s,
                               cur, (const XYZZ<PF>*)prod, oth, rs);
        } else if (ws == 2) {
          if constexpr (PairOps<PF>::ok)
            hipLaunchKernelGGL((ecfft_rsum_kernel<C, PF, 1>), dim3(ecfft_blocks(nb * 2)), dim3(ECFFT_THREADS), 0, s,
                               cur, (const XYZZ<PF>*)prod, oth, rs);
        } else {
          hipLaunchKernelGGL((ecfft_rsum_kernel<C, PF, 0>), dim3(ecfft_blocks(nb)), dim3(ECFFT_THREADS), 0, s, cur,
                             (const XYZZ<PF>*)prod, oth, rs);
        }
        ECG_HIP(hipGetLastError());
        ECG_TRY(kt_end(ctx, "ecfft_stage", s));
        std::swap(cur, oth);
        s0 += d;
      }
      hipLaunchKernelGGL((ecfft_store_kernel<C, PF>), dim3(ecfft_blocks(nb)), dim3(ECFFT_THREADS), 0, s,
                         (const XYZZ<PF>*)cur, (uint32_t)nb, (F*)d_jac);
      ECG_HIP(hipGetLastError());
      return ECG_OK;
    }
  }
  for (uint32_t st = 0; st < log_n; st++) {
    if (abort_cb && abort_cb(user)) {  // ec_fft.rs:112-116, once per round
      (void)hipStreamSynchronize(s);
      return ECG_ABORTED;
    }
    ECG_TRY(kt_begin(ctx, "ecfft_stage", s));
    if constexpr (!std::is_same<PF, F>::value) {
      const size_t stage_lanes = has_glv<C>() ? nb : nb / 2;
      if (win && widen == 4) {
        if constexpr (QuadOps<PF>::ok)
          hipLaunchKernelGGL((ecfft_stage_win_kernel<C, PF, 4>), dim3(ecfft_blocks(4 * stage_lanes)),
                             dim3(ECFFT_THREADS), 0, s, (XYZZ<PF>*)a, (const uint4*)tw, log_n, st, batch,
                             (XYZZ<PF>*)gt);
      } else if (win && pairs) {
        if constexpr (PairOps<PF>::ok)
          hipLaunchKernelGGL((ecfft_stage_win_kernel<C, PF, 1>), dim3(ecfft_blocks(2 * stage_lanes)),
                             dim3(ECFFT_THREADS), 0, s, (XYZZ<PF>*)a, (const uint4*)tw, log_n, st, batch,
                             (XYZZ<PF>*)gt);
      } else if (win) {
        hipLaunchKernelGGL((ecfft_stage_win_kernel<C, PF, 0>), dim3(ecfft_blocks(stage_lanes)),
                           dim3(ECFFT_THREADS), 0, s, (XYZZ<PF>*)a, (const uint4*)tw, log_n, st, batch,
                           (XYZZ<PF>*)gt);
      }
    }
    if (!win)
      hipLaunchKernelGGL((ecfft_stage_kernel<C, PF>), dim3(ecfft_blocks(n / 2)), dim3(ECFFT_THREADS), 0, s,
                         (XYZZ<PF>*)a, (const uint4*)tw, log_n, st, (XYZZ<PF>*)gt);
    ECG_HIP(hipGetLastError());
    ECG_TRY(kt_end(ctx, "ecfft_stage", s));
  }
  hipLaunchKernelGGL((ecfft_store_kernel<C, PF>), dim3(ecfft_blocks(nb)), dim3(ECFFT_THREADS), 0, s,
                     (const XYZZ<PF>*)a, (uint32_t)nb, (F*)d_jac);
  ECG_HIP(hipGetLastError());
  return ECG_OK;
}

template <class C>
static int ecfft_t(ecg_ctx* ctx, void* d_jac, const uint64_t* omega, uint32_t log_n, hipStream_t s,
                   ecg_abort_cb abort_cb, void* user, uint32_t batch) {
  if constexpr (has_rr_form<C>()) {
    if (ecfft_rr_enabled())
      return ecfft_pf<C, FpR<typename RR1of<typename C::FqParams>::Q>>(ctx, d_jac, omega, log_n, s, abort_cb, user,
                                                                         batch);
  }
  if constexpr (has_rr2_form<C>()) {
    if (ecfft_rr_enabled())
      return ecfft_pf<C, FpR2<typename RRof<typename C::FqParams>::Q>>(ctx, d_jac, omega, log_n, s, abort_cb, user,
                                                                         batch);
  }
  return ecfft_pf<C, typename C::Fq>(ctx, d_jac, omega, log_n, s, abort_cb, user, batch);
}

// One curve per translation unit (-DECG_INST=<curve id>, as msm_inst.hip), so
// the four curves' stage kernels build in parallel.
int ecfft_run_0(ecg_ctx*, void*, const uint64_t*, uint32_t, hipStream_t, ecg_abort_cb, void*, uint32_t);
int ecfft_run_1(ecg_ctx*, void*, const uint64_t*, uint32_t, hipStream_t, ecg_abort_cb, void*, uint32_t);
int ecfft_run_2(ecg_ctx*, void*, const uint64_t*, uint32_t, hipStream_t, ecg_abort_cb, void*, uint32_t);
int ecfft_run_3(ecg_ctx*, void*, const uint64_t*, uint32_t, hipStream_t, ecg_abort_cb, void*, uint32_t);

#if ECG_INST == 0
#define ECG_ECFFT_INST_FN ecfft_run_0
using EcfftCurve = BLS12_381;
#elif ECG_INST == 1
#define ECG_ECFFT_INST_FN ecfft_run_1
using EcfftCurve = BN254;
#elif ECG_INST == 2
#define ECG_ECFFT_INST_FN ecfft_run_2
using EcfftCurve = BLS12_381_G2;
#else
#define ECG_ECFFT_INST_FN ecfft_run_3
using EcfftCurve = BN254_G2;
#endif
int ECG_ECFFT_INST_FN(ecg_ctx* ctx, void* d_jac, const uint64_t* omega, uint32_t log_n, hipStream_t s,
                      ecg_abort_cb abort_cb, void* user, uint32_t batch) {
  return ecfft_t<EcfftCurve>(ctx, d_jac, omega, log_n, s, abort_cb, user, batch);
}

#if ECG_INST == 0
}  // namespace ecg

extern "C" int ecg_ec_fft_set_radix(int max_log_radix) {
  if (max_log_radix < 0 || max_log_radix > 8) {
    ecg::set_error("ecg_ec_fft_set_radix: %d is outside 0 (automatic) .. 8", max_log_radix);
    return ECG_ERR_INVALID;
  }
  ecg::ecfft_radix_pin.store(max_log_radix, std::memory_order_relaxed);
  return ECG_OK;
}

namespace ecg {
int ecfft_validate(int curve_id, uint32_t log_n) {
  uint32_t two_adicity = 0;
  ECG_TRY(with_curve(curve_id, "ec_fft", [&](auto c) {
    two_adicity = decltype(c)::FrParams::TWO_ADICITY;
    return ECG_OK;
  }));
  // ec_fft.rs:13 LOG2_MAX_ELEMENTS = 32; the Fr two-adicity bounds it further.
  if (log_n > two_adicity || log_n > 31) {
    set_error("ec_fft: log_n = %u exceeds the supported maximum (two-adicity %u, 2^31 points)", log_n, two_adicity);
    return ECG_ERR_INVALID;
  }
  return ECG_OK;
}

int ecfft_run(ecg_ctx* ctx, int curve_id, void* d_jac, const uint64_t* omega, uint32_t log_n, hipStream_t s,
              ecg_abort_cb abort_cb, void* user, uint32_t batch) {
  ECG_TRY(ecfft_validate(curve_id, log_n));
  if (batch == 0) return ECG_OK;
  switch (curve_id) {  // validated above
    case ECG_CURVE_BLS12_381: return ecfft_run_0(ctx, d_jac, omega, log_n, s, abort_cb, user, batch);
    case ECG_CURVE_BN254: return ecfft_run_1(ctx, d_jac, omega, log_n, s, abort_cb, user, batch);
    case ECG_CURVE_BLS12_381_G2: return ecfft_run_2(ctx, d_jac, omega, log_n, s, abort_cb, user, batch);
    default: return ecfft_run_3(ctx, d_jac, omega, log_n, s, abort_cb, user, batch);
  }
}
#endif

}  // namespace ecg
