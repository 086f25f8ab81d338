// Microbenchmark: VALU integer-multiply roofs on gfx950.
// Measures chip-wide throughput of the candidate multiply primitives for
// multi-precision Montgomery arithmetic:
//   v_mad_u64_u32  (32x32+64 -> 64)     : the int-MAD roof used by DESIGN.md
//   v_mul_lo_u32 + v_mul_hi_u32
//   v_mad_u32_u24 / v_mul_hi_u32_u24
//   v_fma_f64
//   v_add_co_u32 + v_addc_co_u32 (64-bit add)
// Build: hipcc --offload-arch=gfx950 -O3 -o mad_microbench mad_microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8;  // independent chains per lane

__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint64_t acc[CH];
  uint32_t a[CH];
  for (int k = 0; k < CH; k++) { acc[k] = threadIdx.x + k; a[k] = s + k * 7 + threadIdx.x; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) acc[k] = (uint64_t)a[k] * (uint32_t)(acc[k] >> 32) + acc[k];
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; k++) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mullohi(uint64_t* out, uint32_t s) {
  uint32_t lo[CH], hi[CH];
  for (int k = 0; k < CH; k++) { lo[k] = threadIdx.x + k; hi[k] = s + k; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) {
      uint32_t l = lo[k] * hi[k];
      uint32_t h = __umulhi(lo[k], hi[k]);
      lo[k] = l ^ s; hi[k] = h + s;
    }
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; k++) r ^= lo[k] ^ ((uint64_t)hi[k] << 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad24(uint64_t* out, uint32_t s) {
  uint32_t acc[CH], h[CH];
  for (int k = 0; k < CH; k++) { acc[k] = threadIdx.x + k; h[k] = s ^ k; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) {
      uint32_t x = acc[k] & 0xFFFFFF, y = h[k] & 0xFFFFFF;
      uint64_t pr = (uint64_t)x * y; acc[k] = (uint32_t)pr + acc[k];
      h[k] = (uint32_t)(pr >> 32) + h[k];
    }
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; k++) r ^= acc[k] ^ ((uint64_t)h[k] << 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma64(uint64_t* out, uint32_t s) {
  double acc[CH];
  double m = 1.0000001 + s * 1e-12;
  for (int k = 0; k < CH; k++) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) acc[k] = __fma_rn(acc[k], m, 0.5);
  }
  double r = 0;
  for (int k = 0; k < CH; k++) r += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)r;
}

__global__ void k_add64(uint64_t* out, uint32_t s) {
  uint64_t acc[CH];
  uint64_t b = ((uint64_t)s << 32) | 12345;
  for (int k = 0; k < CH; k++) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) acc[k] = acc[k] + (b ^ k);
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; k++) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_add32(uint64_t* out, uint32_t s) {
  uint32_t acc[CH];
  for (int k = 0; k < CH; k++) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) acc[k] = (acc[k] + s) ^ k;
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; k++) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static int run(const char* name, kfn f, double ops_per_iter_chain, uint64_t* d) {
  const int blocks = 256 * 8 * 4, threads = 256;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 3u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  double lane_ops = (double)blocks * threads * ITERS * CH * ops_per_iter_chain;
  printf("%-12s %8.3f ms  %8.2f T lane-ops/s  (%.2f G wave-instr/s per CU)\n", name, best,
         lane_ops / best / 1e9, lane_ops / 64 / best / 1e6 / 256);
  return 0;
}

int main() {
  uint64_t* d;
  CHK(hipMalloc(&d, 256 * 8 * 4 * 256 * sizeof(uint64_t)));
  run("mad_u64_u32", k_mad64, 1, d);
  run("mul_lo+hi", k_mullohi, 2, d);
  run("mul24 lo+hi", k_mad24, 2, d);
  run("fma_f64", k_fma64, 1, d);
  run("add_u64", k_add64, 1, d);
  run("add_u32", k_add32, 1, d);
  CHK(hipFree(d));
  return 0;
}
