// Microbenchmark: cycles per v_mad_u64_u32 for one wave on a SIMD with C
// independent accumulator chains (the column chains of a Montgomery product:
// each mad's 64-bit addend is the previous mad's result).  Tells how many
// interleaved products a latency-bound point operation needs before the
// wave issues at its throughput rate.  One 64-thread workgroup (one wave).
// Build: hipcc --offload-arch=gfx950 -O3 -o mad_latency mad_latency.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int ITERS = 1 << 14;

template <int C>
__global__ void __launch_bounds__(64) k_chain(uint64_t* out, uint32_t s, long long* cyc) {
  uint64_t acc[C];
  uint32_t a[C], b[C];
#pragma unroll
  for (int k = 0; k < C; k++) {
    acc[k] = threadIdx.x + k;
    a[k] = s + 7 * k + threadIdx.x;
    b[k] = s ^ (k * 13);
  }
  const long long t0 = clock64();
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < C; k++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(a[k]), "v"(b[k]));
    }
  }
  const long long t1 = clock64();
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < C; k++) r ^= acc[k];
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int C>
int run(uint64_t* d_out, long long* d_cyc) {
  hipLaunchKernelGGL(k_chain<C>, dim3(1), dim3(64), 0, 0, d_out, 3u, d_cyc);
  CHK(hipGetLastError());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_chain<C>, dim3(1), dim3(64), 0, 0, d_out, 5u, d_cyc);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  long long cyc = 0;
  CHK(hipMemcpy(&cyc, d_cyc, sizeof(cyc), hipMemcpyDeviceToHost));
  const double mads = (double)ITERS * C;
  printf("chains %d: %.2f clock64 ticks per mad, %.3f ns per mad (event), %.2f ns per mad per chain\n", C,
         cyc / mads, ms * 1e6 / mads, ms * 1e6 / ITERS);
  return 0;
}

int main() {
  uint64_t* d_out;
  long long* d_cyc;
  CHK(hipMalloc(&d_out, 64 * sizeof(uint64_t)));
  CHK(hipMalloc(&d_cyc, sizeof(long long)));
  if (run<1>(d_out, d_cyc) || run<2>(d_out, d_cyc) || run<3>(d_out, d_cyc) || run<4>(d_out, d_cyc) ||
      run<6>(d_out, d_cyc) || run<8>(d_out, d_cyc))
    return 1;
  return 0;
}
