// Host-side input preparation of the reference, moved on device (SURVEY
// §8f.3).  Both kernels are HBM-bound byte moves:
//   * density_compact: DensityTracker::generate_exps (ec-gpu-proxy/src/
//     multiexp_cpu.rs:127-138) -- keep exps[i] where bit i of the density
//     bitmap (bitvec Lsb0 over u64 words, multiexp_cpu.rs:117-120) is set.
//     Word popcounts -> exclusive scan -> per-element scatter (32 B / term).
//   * bases_from_ark: arkworks Affine {x, y, infinity: bool} records (104 B
//     for BLS12-381, 72 B for BN254) -> GpuRepr [x, y] with the identity as
//     all zeros (ag-types/src/impls.rs:48-58).
#include <hipcub/hipcub.hpp>

#include "ctx.hpp"

namespace ecg {

constexpr int PREP_THREADS = 256;

__global__ void __launch_bounds__(PREP_THREADS)
    density_popc_kernel(const uint64_t* __restrict__ bits, size_t n, uint32_t* __restrict__ cnt) {
  const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nw = (n + 63) / 64;
  if (w >= nw) return;
  uint64_t word = bits[w];
  const size_t rem = n - w * 64;
  if (rem < 64) word &= (1ull << rem) - 1;  // bits past n are not part of the query
  cnt[w] = (uint32_t)__popcll(word);
}

__global__ void __launch_bounds__(PREP_THREADS)
    density_scatter_kernel(const uint4* __restrict__ exps, const uint64_t* __restrict__ bits, size_t n,
                           const uint32_t* __restrict__ off, uint4* __restrict__ out) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t word = bits[j >> 6];
  const uint32_t b = (uint32_t)(j & 63);
  if (!((word >> b) & 1)) return;
  const size_t pos = off[j >> 6] + (uint32_t)__popcll(word & ((1ull << b) - 1));
  out[2 * pos] = exps[2 * j];
  out[2 * pos + 1] = exps[2 * j + 1];
}

int density_compact(ecg_ctx* ctx, const void* d_exps, const uint64_t* d_bits, size_t n, void* d_out,
                    size_t* out_count, hipStream_t s) {
  *out_count = 0;
  if (n == 0) return ECG_OK;
  if (n > 0xffffffffull) {
    set_error("generate_exps: at most 2^32-1 exponents");
    return ECG_ERR_INVALID;
  }
  const size_t nw = (n + 63) / 64;
  void *cnt, *off, *tmp;
  ECG_TRY(ws_get(ctx, "dens_cnt", nw * 4, &cnt));
  ECG_TRY(ws_get(ctx, "dens_off", nw * 4, &off));
  hipLaunchKernelGGL(density_popc_kernel, dim3((uint32_t)((nw + PREP_THREADS - 1) / PREP_THREADS)),
                     dim3(PREP_THREADS), 0, s, d_bits, n, (uint32_t*)cnt);
  ECG_HIP(hipGetLastError());
  size_t tmp_bytes = 0;
  ECG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, (uint32_t*)cnt, (uint32_t*)off, nw, s));
  ECG_TRY(ws_get(ctx, "dens_tmp", tmp_bytes, &tmp));
  ECG_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (uint32_t*)cnt, (uint32_t*)off, nw, s));
  hipLaunchKernelGGL(density_scatter_kernel, dim3((uint32_t)((n + PREP_THREADS - 1) / PREP_THREADS)),
                     dim3(PREP_THREADS), 0, s, (const uint4*)d_exps, d_bits, n, (const uint32_t*)off,
                     (uint4*)d_out);
  ECG_HIP(hipGetLastError());
  uint32_t last_off = 0, last_cnt = 0;
  ECG_HIP(hipMemcpyAsync(&last_off, (uint32_t*)off + nw - 1, 4, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipMemcpyAsync(&last_cnt, (uint32_t*)cnt + nw - 1, 4, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  *out_count = (size_t)last_off + last_cnt;
  return ECG_OK;
}

// One thread per point; 8-byte words (every field of the record is 8-aligned).
template <int LQ>
__global__ void __launch_bounds__(PREP_THREADS)
    bases_from_ark_kernel(const uint64_t* __restrict__ ark, size_t n, uint64_t* __restrict__ xy) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int STRIDE = 2 * LQ + 1;  // x | y | infinity (bool, padded to 8 B)
  const uint64_t* r = ark + i * STRIDE;
  const bool inf = (r[2 * LQ] & 0xff) != 0;
#pragma unroll
  for (int k = 0; k < 2 * LQ; k++) xy[i * 2 * LQ + k] = inf ? 0ull : r[k];
}

int bases_from_ark(ecg_ctx* ctx, int curve_id, const void* d_ark, size_t n, void* d_xy, hipStream_t s) {
  (void)ctx;
  if (n == 0) return ECG_OK;
  const dim3 grid((uint32_t)((n + PREP_THREADS - 1) / PREP_THREADS));
  const uint64_t* src = (const uint64_t*)d_ark;
  uint64_t* dst = (uint64_t*)d_xy;
  switch (fq_limbs64(curve_id)) {  // G2: x, y in Fq2, then the flag (Affine<G2Config>)
    case 6: hipLaunchKernelGGL(bases_from_ark_kernel<6>, grid, dim3(PREP_THREADS), 0, s, src, n, dst); break;
    case 4: hipLaunchKernelGGL(bases_from_ark_kernel<4>, grid, dim3(PREP_THREADS), 0, s, src, n, dst); break;
    case 12: hipLaunchKernelGGL(bases_from_ark_kernel<12>, grid, dim3(PREP_THREADS), 0, s, src, n, dst); break;
    case 8: hipLaunchKernelGGL(bases_from_ark_kernel<8>, grid, dim3(PREP_THREADS), 0, s, src, n, dst); break;
    default:
      set_error("bases_from_ark: unknown curve_id %d", curve_id);
      return ECG_ERR_INVALID;
  }
  ECG_HIP(hipGetLastError());
  return ECG_OK;
}

}  // namespace ecg
