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
//                      BLS12-381 G1 split into GLV halves k = k1 + k2 LAMBDA
//                      (phi(x, y) = (BETA x, y) = LAMBDA P on G1): the twiddle
//                      product becomes a joint 128-bit ladder over
//                      {P, phi P, P + phi P} -- half the doublings.  Inputs
//                      must be G1 (prime-order subgroup) points, as ark's
//                      G1Projective values are.
//   3. ecfft_stage     log_n launches of n/2 independent radix-2 DIT
//                      butterflies (A, B) -> (A + wB, A - wB), w = 1
//                      butterflies skip the multiply.  G1 points run in the
//                      reduced-radix form of the MSM (curve_rr.hpp: converted
//                      in ecfft_load, back in ecfft_store; ~1.5x faster than
//                      the 32-bit-limb lazy form, which G2 keeps)
//   4. ecfft_store     XYZZ -> normalised Jacobian (x, y, 1) / (0, 1, 0)
#include <cstring>

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

// Twiddle table entry i (2 x uint4): canonical omega^i, or its GLV halves
// (k1 | k2) for curves with the endomorphism.
template <class C>
__global__ void __launch_bounds__(ECFFT_THREADS)
    ecfft_twiddle_kernel(Fp<typename C::FrParams> omega, uint32_t half, uint4* __restrict__ tw) {
  using S = Fp<typename C::FrParams>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  S w = from_mont(fpow_u32(omega, i));
  if constexpr (has_glv<C>()) {
    uint32_t k1[4], k2[4];
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
ECG_DEV XYZZ<PF> glv_joint_mul(const XYZZ<PF>& P, const uint32_t* k1, const uint32_t* k2, XYZZ<PF>* tab) {
  using F = typename C::Fq;
  if (pa_is_zero(P)) return P;
  F beta;
  from_u64_words(beta, C::Gen::BETA);
  XYZZ<PF> phi = P;
  phi.X = pa_mul_const(P.X, beta);
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
      const uint32_t k[4] = {kk.x, kk.y, kk.z, kk.w};
      typename C::Fq beta;
      from_u64_words(beta, C::Gen::BETA);
      XYZZ<PF> Bh = B;
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

static uint32_t ecfft_pairs_max() {  // A/B: ECG_ECFFT_PAIRS = 0 / 1 (single lanes), 2 (pairs), 4 (quads)
  static const uint32_t v = [] {
    const char* e = getenv("ECG_ECFFT_PAIRS");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 4u;
  }();
  return v;
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
  return with_curve(curve_id, "ec_fft",
                    [&](auto c) { return ecfft_t<decltype(c)>(ctx, d_jac, omega, log_n, s, abort_cb, user, batch); });
}

}  // namespace ecg
