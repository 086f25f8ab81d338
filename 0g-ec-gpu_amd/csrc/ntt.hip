// Radix-2^DEG Stockham NTT over the scalar fields (BLS12-381 Fr, BN254 Fr).
//
// Replaces FIELD_radix_fft (ag-build/cl/fft.cl:4-68) and its host driver
// SingleFftKernel::radix_fft (ec-gpu-proxy/src/fft.rs:50-135).  Same
// decomposition (Stockham autosort, natural order in and out, passes of up to
// 2^8 points), re-designed for gfx950:
//
//  * A workgroup owns G = TILE >> DEG consecutive Stockham groups (TILE = 1024
//    elements = 32 KiB of LDS).  Lanes walk the G groups fastest, so every
//    global read of x[g + i*t] is a G*32-byte contiguous run and the writes
//    are contiguous runs of min(p, G)*32 bytes (first pass: whole 2^DEG*32 B
//    groups).  The reference uses one group per block (fft.rs:104-118).
//  * No per-thread exponentiation: the reference computes twiddle^counts with
//    FIELD_pow_lookup + FIELD_pow per thread (fft.cl:39-45, about 4x the
//    butterfly work).  Here inter-pass twiddles w^e (e < n) come from two
//    precomputed tables, w^e = T_hi[e >> S] * T_lo[e & (2^S-1)] (2 muls per
//    element, L2-resident), and the in-group roots pq[] sit in LDS.
//  * Elements live in LDS as two 16-byte planes (conflict-free ds_read_b128
//    for consecutive indices); DIF butterflies run DEG rounds in LDS and the
//    final bit-reversal is folded into the output index (fft.cl:64-67).
//  * Values stay fully reduced (< r) so the output bytes equal serial_fft's.
#include <cstring>

#include "ctx.hpp"
#include "field.hpp"

namespace ecg {

constexpr int NTT_THREADS = 256;
constexpr int NTT_TILE_LOG = 10;  // 1024 elements per workgroup tile
constexpr int NTT_MAX_DEG = 8;    // radix-256 passes (MAX_LOG2_RADIX, fft.rs:15)
constexpr int NTT_LO_BITS = 12;   // twiddle split table size 2^12

template <class F>
struct LdsPlanes {
  uint4* p0;
  uint4* p1;
  ECG_DEV F get(uint32_t i) const {
    uint4 a = p0[i], b = p1[i];
    F r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
  }
  ECG_DEV void put(uint32_t i, const F& v) const {
    p0[i] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
    p1[i] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
  }
};

ECG_DEV uint32_t bitrev(uint32_t x, int bits) { return __builtin_bitreverse32(x) >> (32 - bits); }

// One Stockham pass: groups g in [blockIdx.x*G, +G), G = 2^log_g.
//   u[i] = x[g + i*t] * w^((n >> (lgp+DEG)) * k * i),  k = g mod 2^lgp, t = n >> DEG
//   v = DFT_{2^DEG}(u)  (root w^(n >> DEG))
//   y[(g - k)*2^DEG + k + j*2^lgp] = v[j]
template <class P, int DEG>
__global__ void __launch_bounds__(NTT_THREADS)
    ntt_pass_kernel(const Fp<P>* __restrict__ x, Fp<P>* __restrict__ y, const Fp<P>* __restrict__ pq,
                    uint32_t pq_shift, const Fp<P>* __restrict__ tw_lo, const Fp<P>* __restrict__ tw_hi,
                    uint32_t log_n, uint32_t lgp, uint32_t log_g) {
  using F = Fp<P>;
  static_assert(F::L == 8, "NTT tiles assume 32-byte scalar-field elements");
  constexpr uint32_t R = 1u << DEG;
  extern __shared__ uint4 smem[];
  const uint32_t G = 1u << log_g;
  const uint32_t E = G << DEG;
  LdsPlanes<F> U{smem, smem + E};
  LdsPlanes<F> W{smem + 2 * E, smem + 2 * E + R / 2};

  const uint64_t n = 1ull << log_n;
  const uint64_t t = n >> DEG;
  const uint64_t p = 1ull << lgp;
  const uint64_t g0 = (uint64_t)blockIdx.x << log_g;
  const uint32_t tid = threadIdx.x;

  // in-group roots w_{2^DEG}^j, j < R/2 (pq is for 2^max_deg: stride pq_shift)
  for (uint32_t j = tid; j < R / 2; j += NTT_THREADS) W.put(j, load(&pq[(uint64_t)j << pq_shift]));

  // load (+ inter-pass twiddle), lanes walk the G groups fastest
  const uint32_t s_tw_log = log_n - lgp - DEG;  // n >> (lgp + DEG) = 2^s_tw_log
  for (uint32_t f = tid; f < E; f += NTT_THREADS) {
    const uint32_t gi = f & (G - 1), i = f >> log_g;
    const uint64_t g = g0 + gi;
    F v = load(&x[g + (uint64_t)i * t]);
    if (lgp != 0) {
      const uint64_t k = g & (p - 1);
      const uint64_t e = (k * i) << s_tw_log;  // < n
      if (e != 0) {
        F w = fmul(load(&tw_hi[e >> NTT_LO_BITS]), load(&tw_lo[e & ((1u << NTT_LO_BITS) - 1)]));
        v = fmul(v, w);
      }
    }
    U.put((gi << DEG) + i, v);
  }
  __syncthreads();

  // DIF radix-2 rounds (fft.cl:48-62)
#pragma unroll 1
  for (int rnd = 0; rnd < DEG; rnd++) {
    const uint32_t bit = (R / 2) >> rnd;
    for (uint32_t f = tid; f < E / 2; f += NTT_THREADS) {
      const uint32_t gi = f >> (DEG - 1), b = f & (R / 2 - 1);
      const uint32_t di = b & (bit - 1);
      const uint32_t i0 = (gi << DEG) + (b << 1) - di, i1 = i0 + bit;
      F u0 = U.get(i0), u1 = U.get(i1);
      F s = fadd(u0, u1);
      F d = fsub(u0, u1);
      if (di != 0) d = fmul(d, W.get(di << rnd));
      U.put(i0, s);
      U.put(i1, d);
    }
    __syncthreads();
  }

  // store: y[(g - k)*R + k + j*p] = u[bitrev(j)], lanes walk min(p, G) fastest
  const uint32_t lpp = lgp < log_g ? lgp : log_g;  // log2 min(p, G)
  const uint32_t pp = 1u << lpp;
  for (uint32_t f = tid; f < E; f += NTT_THREADS) {
    const uint32_t kk = f & (pp - 1);
    const uint32_t j = (f >> lpp) & (R - 1);
    const uint32_t gh = f >> (lpp + DEG);
    const uint32_t gi = (gh << lpp) + kk;
    const uint64_t g = g0 + gi;
    const uint64_t k = g & (p - 1);
    F v = U.get((gi << DEG) + bitrev(j, DEG));
    store(&y[((g - k) << DEG) + k + (uint64_t)j * p], v);
  }
}

// out[j] = w^(j << shift), j < count  (w given by value, Montgomery)
template <class P>
__global__ void ntt_powers_kernel(Fp<P> w, uint32_t shift, uint64_t count, Fp<P>* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  // base = w^(2^shift)
  Fp<P> base = w;
  for (uint32_t s = 0; s < shift; s++) base = fsqr(base);
  Fp<P> r = Fp<P>::one();
  uint64_t e = j;
  while (e) {
    if (e & 1) r = fmul(r, base);
    e >>= 1;
    if (e) base = fsqr(base);
  }
  store(&out[j], r);
}

template <class P, int DEG>
static hipError_t launch_pass(const void* x, void* y, const void* pq, uint32_t pq_shift, const void* tw_lo,
                              const void* tw_hi, uint32_t log_n, uint32_t lgp, hipStream_t s) {
  using F = Fp<P>;
  uint32_t log_g = NTT_TILE_LOG - DEG;
  const uint32_t log_groups = log_n - DEG;
  if (log_g > log_groups) log_g = log_groups;
  const uint64_t blocks = 1ull << (log_groups - log_g);
  const size_t lds = ((size_t)2 << (log_g + DEG)) * sizeof(uint4) + (size_t)(1u << DEG) * sizeof(uint4);
  hipLaunchKernelGGL((ntt_pass_kernel<P, DEG>), dim3((uint32_t)blocks), dim3(NTT_THREADS), lds, s,
                     (const F*)x, (F*)y, (const F*)pq, pq_shift, (const F*)tw_lo, (const F*)tw_hi, log_n, lgp,
                     log_g);
  return hipGetLastError();
}

template <class P>
static hipError_t launch_pass_deg(int deg, const void* x, void* y, const void* pq, uint32_t pq_shift,
                                  const void* tw_lo, const void* tw_hi, uint32_t log_n, uint32_t lgp,
                                  hipStream_t s) {
  switch (deg) {
    case 1: return launch_pass<P, 1>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 2: return launch_pass<P, 2>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 3: return launch_pass<P, 3>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 4: return launch_pass<P, 4>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 5: return launch_pass<P, 5>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 6: return launch_pass<P, 6>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 7: return launch_pass<P, 7>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    case 8: return launch_pass<P, 8>(x, y, pq, pq_shift, tw_lo, tw_hi, log_n, lgp, s);
    default: return hipErrorInvalidValue;
  }
}

template <class P>
static int ntt_run_t(ecg_ctx* ctx, int field_id, void* d_data, const uint64_t* omega, uint32_t log_n,
                     hipStream_t s, ecg_abort_cb abort_cb, void* user) {
  using F = Fp<P>;
  if (log_n == 0) {
    // fft.rs:68-70: pq has length 0 -> the reference panics on pq[0]
    set_error("radix_fft: log_n must be >= 1");
    return ECG_ERR_INVALID;
  }
  if (log_n > (uint32_t)P::TWO_ADICITY || log_n > 32) {
    set_error("radix_fft: log_n %u exceeds the field's two-adicity", log_n);
    return ECG_ERR_INVALID;
  }
  const uint64_t n = 1ull << log_n;
  const uint32_t max_deg = log_n < (uint32_t)NTT_MAX_DEG ? log_n : NTT_MAX_DEG;
  const uint32_t lo_bits = NTT_LO_BITS;
  const uint64_t lo_cnt = 1ull << lo_bits;
  const uint64_t hi_cnt = n > lo_cnt ? (n >> lo_bits) : 1;
  const uint64_t pq_cnt = 1ull << (max_deg - 1);

  void *scratch, *tables;
  ECG_TRY(ws_get(ctx, "ntt_scratch", n * sizeof(F), &scratch));
  ECG_TRY(ws_get(ctx, "ntt_tables", (pq_cnt + lo_cnt + hi_cnt) * sizeof(F), &tables));
  F* pq = (F*)tables;
  F* tw_lo = pq + pq_cnt;
  F* tw_hi = tw_lo + lo_cnt;

  const bool cached = ctx->tw_fid == field_id && ctx->tw_log_n == log_n &&
                      memcmp(ctx->tw_omega, omega, sizeof(ctx->tw_omega)) == 0;
  if (!cached) {
    F w;
    memcpy(w.v, omega, sizeof(w.v));
    // pq[j] = w^(j * (n >> max_deg)) (fft.rs:68-78); tw_lo[j] = w^j; tw_hi[j] = w^(j << lo_bits)
    hipLaunchKernelGGL(ntt_powers_kernel<P>, dim3((uint32_t)((pq_cnt + 255) / 256)), dim3(256), 0, s, w,
                       log_n - max_deg, pq_cnt, pq);
    hipLaunchKernelGGL(ntt_powers_kernel<P>, dim3((uint32_t)((lo_cnt + 255) / 256)), dim3(256), 0, s, w, 0u,
                       lo_cnt, tw_lo);
    hipLaunchKernelGGL(ntt_powers_kernel<P>, dim3((uint32_t)((hi_cnt + 255) / 256)), dim3(256), 0, s, w,
                       lo_bits, hi_cnt, tw_hi);
    ECG_HIP(hipGetLastError());
    ctx->tw_fid = field_id;
    ctx->tw_log_n = log_n;
    memcpy(ctx->tw_omega, omega, sizeof(ctx->tw_omega));
  }

  kt_reset(ctx, "ntt_pass");
  void* src = d_data;
  void* dst = scratch;
  uint32_t lgp = 0;
  while (lgp < log_n) {
    if (abort_cb && abort_cb(user)) return ECG_ABORTED;  // fft.rs:94-98
    const uint32_t deg = (log_n - lgp) < max_deg ? (log_n - lgp) : max_deg;
    ECG_TRY(kt_begin(ctx, "ntt_pass", s));
    ECG_HIP(launch_pass_deg<P>((int)deg, src, dst, pq, max_deg - deg, tw_lo, tw_hi, log_n, lgp, s));
    ECG_TRY(kt_end(ctx, "ntt_pass", s));
    lgp += deg;
    void* tmp = src;
    src = dst;
    dst = tmp;
  }
  if (src != d_data) ECG_HIP(hipMemcpyAsync(d_data, src, n * sizeof(F), hipMemcpyDeviceToDevice, s));
  return ECG_OK;
}

int ntt_validate(int field_id, uint32_t log_n) {
  uint32_t adic;
  switch (field_id) {
    case ECG_FIELD_BLS12_381_FR: adic = params::bls12_381_fr::TWO_ADICITY; break;
    case ECG_FIELD_BN254_FR: adic = params::bn254_fr::TWO_ADICITY; break;
    default:
      set_error("radix_fft: field_id %d is not an FFT-friendly scalar field", field_id);
      return ECG_ERR_INVALID;
  }
  if (log_n == 0) {
    set_error("radix_fft: log_n must be >= 1");  // the reference panics (fft.rs:68-70)
    return ECG_ERR_INVALID;
  }
  if (log_n > adic || log_n > 32) {
    set_error("radix_fft: log_n %u exceeds the field's two-adicity %u", log_n, adic);
    return ECG_ERR_INVALID;
  }
  return ECG_OK;
}

int ntt_run(ecg_ctx* ctx, int field_id, void* d_data, const uint64_t* omega, uint32_t log_n, hipStream_t s,
            ecg_abort_cb abort_cb, void* user) {
  switch (field_id) {
    case ECG_FIELD_BLS12_381_FR:
      return ntt_run_t<params::bls12_381_fr>(ctx, field_id, d_data, omega, log_n, s, abort_cb, user);
    case ECG_FIELD_BN254_FR:
      return ntt_run_t<params::bn254_fr>(ctx, field_id, d_data, omega, log_n, s, abort_cb, user);
    default:
      set_error("radix_fft: field_id %d is not an FFT-friendly scalar field", field_id);
      return ECG_ERR_INVALID;
  }
}

}  // namespace ecg
