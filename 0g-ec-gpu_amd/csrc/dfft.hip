// One NTT of size n = 2^log_n split over T ranks: the four-step
// decomposition that parallel_fft restates on CPU threads (ec-gpu-proxy/src/
// fft_cpu.rs:59-111), re-laid-out for block-distributed data and RCCL
// all-to-all exchanges over xGMI.
//
// With m = n / T and seg = m / T, input index j = j1*m + j2 (rank j1 holds the
// block a[j1*m .. (j1+1)*m)) and output index k = k1 + T*k2:
//   out[k1 + T k2] = sum_j2 w_m^(j2 k2) * [ w^(j2 k1) * sum_j1 z^(j1 k1) a[j1 m + j2] ]
// with w_m = w^T and z = w^m (a T-th root of unity).
//   all-to-all #1   rank q receives, from every rank s, a[s m + q seg + i], i < seg
//   stage1          T-point DFT over s, twiddle w^(j2 k1)      -> [k1][i] segments
//   all-to-all #2   rank k1 receives y[k1][j2] for every j2 (contiguous in j2)
//   local NTT       m points with w^T (ntt_run)               -> out[k1 + T k2]
//   all-to-all #3   rank r receives out[r m + T i + k1] as [k1][i]
//   stage3          [T][seg] -> [seg][T] interleave            -> block r of out
// Exchanges are equal-split (seg elements per peer).  Stages 1/3 are
// HBM-bound element moves plus ~T + log n Fr products per T elements.
#include <cstring>

#include "ctx.hpp"
#include "field.hpp"

namespace ecg {

constexpr int DFFT_THREADS = 256;
constexpr uint32_t DFFT_MAX_T = 16;

template <class P, uint32_t T>
__global__ void __launch_bounds__(DFFT_THREADS)
    dfft_stage1_kernel(const Fp<P>* __restrict__ in, Fp<P>* __restrict__ out, Fp<P> omega, uint32_t rank,
                       size_t seg, uint32_t log_m) {
  using F = Fp<P>;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= seg) return;
  const size_t j2 = (size_t)rank * seg + i;
  F x[T];
  for (uint32_t s = 0; s < T; s++) x[s] = load(&in[(size_t)s * seg + i]);
  // z = w^m (T-th root), w^j2 (j2 < m <= 2^31)
  F z = omega;
  for (uint32_t b = 0; b < log_m; b++) z = fsqr(z);
  F wj = fpow_u32(omega, (uint32_t)j2);
  F zk = F::one();   // z^k1
  F tw = F::one();   // w^(j2 k1)
  for (uint32_t k1 = 0; k1 < T; k1++) {
    // y = sum_s x[s] z^(s k1), Horner in z^k1 from the top
    F y = x[T - 1];
    if constexpr (T > 1) {
      for (int s = (int)T - 2; s >= 0; s--) y = fadd(fmul(y, zk), x[s]);
    }
    store(&out[(size_t)k1 * seg + i], fmul(y, tw));
    zk = fmul(zk, z);
    tw = fmul(tw, wj);
  }
}

__global__ void __launch_bounds__(DFFT_THREADS)
    dfft_stage3_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t T, size_t seg) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // output element
  if (e >= seg * T) return;
  const size_t i = e / T;
  const uint32_t k1 = (uint32_t)(e % T);
  const size_t src = (size_t)k1 * seg + i;
  out[2 * e] = in[2 * src];
  out[2 * e + 1] = in[2 * src + 1];
}

static int dfft_check(int field_id, uint32_t T, uint32_t log_n, uint32_t* log_t) {
  if (field_id != ECG_FIELD_BLS12_381_FR && field_id != ECG_FIELD_BN254_FR) {
    set_error("distributed fft: unsupported field_id %d", field_id);
    return ECG_ERR_INVALID;
  }
  if (T == 0 || (T & (T - 1)) || T > DFFT_MAX_T) {
    set_error("distributed fft: rank count %u must be a power of two <= %u", T, DFFT_MAX_T);
    return ECG_ERR_INVALID;
  }
  uint32_t lt = 0;
  while ((1u << lt) < T) lt++;
  if (log_n < 2 * lt + 1) {  // seg >= 1 and m >= 2 (the local NTT rejects log 0)
    set_error("distributed fft: 2^%u points is too small for %u ranks", log_n, T);
    return ECG_ERR_INVALID;
  }
  ECG_TRY(ntt_validate(field_id, log_n));
  *log_t = lt;
  return ECG_OK;
}

template <class P>
static int dfft_stage1_t(const void* d_in, void* d_out, const uint64_t* omega, uint32_t T, uint32_t rank,
                         uint32_t log_n, uint32_t log_t, hipStream_t s) {
  Fp<P> om;
  memcpy(om.v, omega, sizeof(om.v));
  const size_t seg = (size_t)1 << (log_n - 2 * log_t);
  const dim3 grid((uint32_t)((seg + DFFT_THREADS - 1) / DFFT_THREADS)), blk(DFFT_THREADS);
  const Fp<P>* in = (const Fp<P>*)d_in;
  Fp<P>* out = (Fp<P>*)d_out;
  const uint32_t lm = log_n - log_t;
  switch (T) {
    case 1: hipLaunchKernelGGL((dfft_stage1_kernel<P, 1>), grid, blk, 0, s, in, out, om, rank, seg, lm); break;
    case 2: hipLaunchKernelGGL((dfft_stage1_kernel<P, 2>), grid, blk, 0, s, in, out, om, rank, seg, lm); break;
    case 4: hipLaunchKernelGGL((dfft_stage1_kernel<P, 4>), grid, blk, 0, s, in, out, om, rank, seg, lm); break;
    case 8: hipLaunchKernelGGL((dfft_stage1_kernel<P, 8>), grid, blk, 0, s, in, out, om, rank, seg, lm); break;
    default: hipLaunchKernelGGL((dfft_stage1_kernel<P, 16>), grid, blk, 0, s, in, out, om, rank, seg, lm); break;
  }
  ECG_HIP(hipGetLastError());
  return ECG_OK;
}

int dfft_stage1(int field_id, const void* d_in, void* d_out, const uint64_t* omega, uint32_t T, uint32_t rank,
                uint32_t log_n, hipStream_t s) {
  uint32_t lt;
  ECG_TRY(dfft_check(field_id, T, log_n, &lt));
  if (rank >= T) {
    set_error("distributed fft: rank %u out of range [0, %u)", rank, T);
    return ECG_ERR_INVALID;
  }
  if (field_id == ECG_FIELD_BLS12_381_FR)
    return dfft_stage1_t<params::bls12_381_fr>(d_in, d_out, omega, T, rank, log_n, lt, s);
  return dfft_stage1_t<params::bn254_fr>(d_in, d_out, omega, T, rank, log_n, lt, s);
}

int dfft_stage3(const void* d_in, void* d_out, uint32_t T, uint32_t log_n, hipStream_t s) {
  uint32_t lt;
  ECG_TRY(dfft_check(ECG_FIELD_BLS12_381_FR, T, log_n, &lt));
  const size_t seg = (size_t)1 << (log_n - 2 * lt);
  const size_t m = seg * T;
  hipLaunchKernelGGL(dfft_stage3_kernel, dim3((uint32_t)((m + DFFT_THREADS - 1) / DFFT_THREADS)),
                     dim3(DFFT_THREADS), 0, s, (const uint4*)d_in, (uint4*)d_out, T, seg);
  ECG_HIP(hipGetLastError());
  return ECG_OK;
}

// w^T in Montgomery form (host): omega of the local m-point NTT.
static void pow2k_host(int field_id, const uint64_t* omega, uint32_t k, uint64_t* out);

// Every local failure (arguments, workspace, the local NTT, abort_cb) is
// exchanged (comm_agree) before the all-to-all that would otherwise leave the
// peers waiting for this rank: once before the first, once before the last.
int dfft_run(ecg_ctx* ctx, int field_id, void* d_local, const uint64_t* omega, uint32_t log_n, hipStream_t s,
             ecg_abort_cb abort_cb, void* user) {
  const uint32_t T = (uint32_t)ctx->comm_size, rank = (uint32_t)ctx->comm_rank;
  uint32_t lt = 0;
  void* b = nullptr;
  int rc = ECG_OK;
  if (!d_local || !omega) {
    set_error("ecg_fft_dist: null pointer");
    rc = ECG_ERR_INVALID;
  } else {
    rc = dfft_check(field_id, T, log_n, &lt);
  }
  const size_t m = rc == ECG_OK ? (size_t)1 << (log_n - lt) : 0;
  if (rc == ECG_OK) rc = ws_get(ctx, "dfft_b", m * 32, &b);
  if (rc == ECG_OK && abort_cb && abort_cb(user)) rc = ECG_ABORTED;  // fft.rs:94-98
  const uint64_t agree[2] = {(uint64_t)(uint32_t)field_id, log_n};
  ECG_TRY(comm_agree(ctx, rc, agree, 2, "ecg_fft_dist", s));
  const size_t seg_bytes = (m / T) * 32;
  ECG_TRY(comm_alltoall(ctx, d_local, b, seg_bytes, s));
  ECG_TRY(dfft_stage1(field_id, b, d_local, omega, T, rank, log_n, s));
  ECG_TRY(comm_alltoall(ctx, d_local, b, seg_bytes, s));
  uint64_t om_t[4];
  pow2k_host(field_id, omega, lt, om_t);
  rc = ntt_run(ctx, field_id, b, om_t, log_n - lt, s, nullptr, nullptr);
  if (rc == ECG_OK && abort_cb && abort_cb(user)) rc = ECG_ABORTED;
  ECG_TRY(comm_agree(ctx, rc, agree, 2, "ecg_fft_dist", s));
  ECG_TRY(comm_alltoall(ctx, b, d_local, seg_bytes, s));
  ECG_TRY(dfft_stage3(d_local, b, T, log_n, s));
  ECG_HIP(hipMemcpyAsync(d_local, b, m * 32, hipMemcpyDeviceToDevice, s));
  return ECG_OK;
}

}  // namespace ecg

#include "host_field.hpp"

namespace ecg {
static void pow2k_host(int field_id, const uint64_t* omega, uint32_t k, uint64_t* out) {
  if (field_id == ECG_FIELD_BLS12_381_FR) {
    host::HFp<params::bls12_381_fr> w;
    memcpy(w.v, omega, sizeof(w.v));
    for (uint32_t i = 0; i < k; i++) w = host::hmul(w, w);
    memcpy(out, w.v, sizeof(w.v));
  } else {
    host::HFp<params::bn254_fr> w;
    memcpy(w.v, omega, sizeof(w.v));
    for (uint32_t i = 0; i < k; i++) w = host::hmul(w, w);
    memcpy(out, w.v, sizeof(w.v));
  }
}
}  // namespace ecg
