// Dependent-chain issue microbenchmark (tools only): how many cycles a wave64
// v_mad_u64_u32 costs when the stream has only K independent accumulator
// chains (K = 1, 2, 4) at 1-4 waves per SIMD, and the same for the reduced-
// radix product's column end (mads, then the digit v_mul_lo -> v_and -> mad ->
// 64-bit shift, every step dependent on the previous) at K = 2 and 4 chains.
// The accumulation's products pair two chains (rr_mul2); this measures what
// that pairing leaves on the table.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o dep_bench dep_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

__device__ __forceinline__ void mad2(uint64_t& a0, uint64_t& a1, uint32_t x, uint32_t y) {
  uint64_t c0, c1;
  asm volatile("v_mad_u64_u32 %0, %2, %4, %5, %0\n\tv_mad_u64_u32 %1, %3, %4, %5, %1"
               : "+v"(a0), "+v"(a1), "=&s"(c0), "=&s"(c1) : "v"(x), "v"(y));
}
__device__ __forceinline__ void mad2p(uint64_t& a0, uint32_t m0, uint64_t& a1, uint32_t m1, uint32_t p) {
  uint64_t c0, c1;
  asm volatile("v_mad_u64_u32 %0, %2, %4, %6, %0\n\tv_mad_u64_u32 %1, %3, %5, %6, %1"
               : "+v"(a0), "+v"(a1), "=&s"(c0), "=&s"(c1) : "v"(m0), "v"(m1), "v"(p));
}

// K chains (K even) of L mads per column, mads paired two chains per asm
// statement as in rr_mul2, then (END) every chain's column end
template <int K, int L, bool END>
__global__ void __launch_bounds__(256) k_chain(uint64_t* out, uint32_t s) {
  uint64_t a[K];
#pragma unroll
  for (int k = 0; k < K; k++) a[k] = s + k;
  const uint32_t x = threadIdx.x | 1, y = s | 3, inv = s * 7 + 1, p0 = s * 5 + 3;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int l = 0; l < L; l++)
#pragma unroll
      for (int k = 0; k < K; k += 2) mad2(a[k], a[k + 1], x, y);
    if (END) {
#pragma unroll
      for (int k = 0; k < K; k += 2) {
        const uint32_t m0 = ((uint32_t)a[k] * inv) & 0x1fffffffu, m1 = ((uint32_t)a[k + 1] * inv) & 0x1fffffffu;
        mad2p(a[k], m0, a[k + 1], m1, p0);
        a[k] >>= 29;
        a[k + 1] >>= 29;
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < K; k++) r ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kern_t)(uint64_t*, uint32_t);

int main() {
  // instr = VALU instructions per trip (a column end: mul_lo, and, mad, 64-bit shift)
  struct { const char* name; kern_t k; int instr; } ks[] = {
      {"mad ILP2", k_chain<2, 8, false>, 16},
      {"mad ILP4", k_chain<4, 4, false>, 16}, {"mad ILP8", k_chain<8, 2, false>, 16},
      {"col9 x2 chains", k_chain<2, 9, true>, 2 * 9 + 2 * 4}, {"col9 x4 chains", k_chain<4, 9, true>, 4 * 9 + 4 * 4},
      {"col13 x2 chains", k_chain<2, 13, true>, 2 * 13 + 2 * 4}, {"col18 x2 chains", k_chain<2, 18, true>, 2 * 18 + 2 * 4},
      {"col26 x2 chains", k_chain<2, 26, true>, 2 * 26 + 2 * 4},
  };
  uint64_t* out;
  CHK(hipMalloc(&out, sizeof(uint64_t) << 22));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int ncu = 256;
  for (int wps : {1, 2, 3, 4}) {
    const int blocks = ncu * wps, threads = 256;  // one wave per SIMD per block
    for (auto& k : ks) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; rep++) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      const double winstr = (double)blocks * threads / 64 * ITERS * k.instr;
      const double cyc = best * 1e-3 * 2.4e9 * ncu * 4 / winstr;  // SIMD cycles per wave-instruction at 2.4 GHz
      printf("waves/SIMD %d  %-16s %8.3f ms  %6.2f SIMD-cyc per wave-instr (2.4 GHz)\n", wps, k.name, best, cyc);
    }
  }
  return 0;
}
