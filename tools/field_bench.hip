// Field-multiply microbenchmark + correctness probe (tools only, not product).
// Times Montgomery multiplication throughput for the product-scanning asm
// variant (ecg::fmul) and the portable CIOS variant (ecg::fmul_cios) on
// BLS12-381 Fr (8x32 limbs) and Fq (12x32 limbs), and checks every GPU result
// against the CPU oracle (oracle/build/liboracle.so, dlopen'ed).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../0g-ec-gpu_amd/csrc/field.hpp"

using namespace ecg;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int ITERS = 256;
constexpr int CH = 2;

template <class F, int V>
__global__ void k_chain(const F* x, const F* y, F* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  F a[CH], b = load(&y[t]);
  for (int k = 0; k < CH; k++) a[k] = load(&x[(t + k) % n]);
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++)
      a[k] = V == 0 ? fmul(a[k], b) : V == 1 ? fmul_cios(a[k], b) : V == 2 ? fmul_x4(a[k], b) : fmul_ilp(a[k], b);
  }
  F r = a[0];
  for (int k = 1; k < CH; k++) r = fadd(r, a[k]);
  store(&out[t], r);
}

// Same chain, but one chain per thread and occupancy forced by dynamic LDS:
// waves/SIMD = 8 / (blocks of 256 per CU limited by LDS).
template <class F, int V>
__global__ void k_chain_occ(const F* x, const F* y, F* out, int n) {
  extern __shared__ uint32_t lds_pad[];
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  F a = load(&x[t]), b = load(&y[t]);
  for (int i = 0; i < ITERS; i++) a = V == 3 ? fmul_ilp(a, b) : fmul(a, b);
  if (threadIdx.x == 1023) lds_pad[0] = a.v[0];  // keep the LDS allocation
  store(&out[t], a);
}

template <class F>
__global__ void k_once(const F* x, const F* y, F* o0, F* o1, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  F a = load(&x[t]), b = load(&y[t]);
  store(&o0[t], fmul(a, b));
  store(&o1[t], fmul_cios(a, b));
  if (!feq(fmul_x4(a, b), fmul_cios(a, b))) o1[t].v[0] ^= 1;
  if (!feq(fmul_ilp(a, b), fmul_cios(a, b))) o1[t].v[1] ^= 1;
}

typedef void (*orc_fmul_t)(int, uint64_t*, const uint64_t*, const uint64_t*);

static uint64_t rng_state = 0x1234567;
static uint64_t rnd() {
  rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17;
  return rng_state;
}

template <class F>
static void bench(const char* name, int fid, orc_fmul_t orc) {
  constexpr int N = F::N;
  const int n = 256 * 256 * 8;
  std::vector<F> hx(n), hy(n);
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < F::L; k++) { hx[i].v[k] = (uint32_t)rnd(); hy[i].v[k] = (uint32_t)rnd(); }
    hx[i].v[F::L - 1] &= 0x0fffffff; hy[i].v[F::L - 1] &= 0x0fffffff;  // < p for all our moduli
  }
  // edge values: 0, p-1
  for (int k = 0; k < F::L; k++) { hx[0].v[k] = 0; hx[1].v[k] = F::p32(k); hy[1].v[k] = F::p32(k); }
  hx[1].v[0] -= 1; hy[1].v[0] -= 1;
  F *dx, *dy, *d0, *d1;
  CHK(hipMalloc(&dx, n * sizeof(F))); CHK(hipMalloc(&dy, n * sizeof(F)));
  CHK(hipMalloc(&d0, n * sizeof(F))); CHK(hipMalloc(&d1, n * sizeof(F)));
  CHK(hipMemcpy(dx, hx.data(), n * sizeof(F), hipMemcpyHostToDevice));
  CHK(hipMemcpy(dy, hy.data(), n * sizeof(F), hipMemcpyHostToDevice));
  k_once<F><<<n / 256, 256>>>(dx, dy, d0, d1, n);
  CHK(hipDeviceSynchronize());
  std::vector<F> r0(n), r1(n);
  CHK(hipMemcpy(r0.data(), d0, n * sizeof(F), hipMemcpyDeviceToHost));
  CHK(hipMemcpy(r1.data(), d1, n * sizeof(F), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < n; i++) {
    uint64_t e[N];
    if (orc && i < 4096) {
      orc(fid, e, reinterpret_cast<const uint64_t*>(&hx[i]), reinterpret_cast<const uint64_t*>(&hy[i]));
      if (memcmp(e, &r0[i], sizeof(F)) != 0) bad++;
    }
    if (memcmp(&r0[i], &r1[i], sizeof(F)) != 0) bad++;
  }
  printf("%s correctness: %s (%d mismatches)\n", name, bad ? "FAIL" : "ok", bad);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  float best[4] = {1e30f, 1e30f, 1e30f, 1e30f};
  for (int rep = 0; rep < 6; rep++) {
    for (int v = 0; v < 4; v++) {  // interleaved rounds: A/B in one process
      CHK(hipEventRecord(a));
      if (v == 0) k_chain<F, 0><<<n / 256, 256>>>(dx, dy, d0, n);
      else if (v == 1) k_chain<F, 1><<<n / 256, 256>>>(dx, dy, d1, n);
      else if (v == 2) k_chain<F, 2><<<n / 256, 256>>>(dx, dy, d1, n);
      else k_chain<F, 3><<<n / 256, 256>>>(dx, dy, d1, n);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms; CHK(hipEventElapsedTime(&ms, a, b));
      if (ms < best[v]) best[v] = ms;
    }
  }
  for (int v = 0; v < 4; v++) {
    double muls = (double)n * ITERS * CH;
    printf("  %-6s %s: %8.3f ms  %8.2f G mul/s\n", name,
           v == 0 ? "fips-asm-x1" : v == 1 ? "cios-c++" : v == 2 ? "fips-asm-x4" : "fips-ilp2", best[v],
           muls / best[v] / 1e6);
  }
  // throughput vs occupancy (1 chain per thread): LDS per 256-thread block sets blocks/CU
  for (int wps : {1, 2, 3, 4, 8}) {
    size_t lds = wps >= 8 ? 0 : (160 * 1024) / wps - 256;  // blocks per CU = wps (each block = 1 wave/SIMD)
    float bst[2] = {1e30f, 1e30f};
    for (int rep = 0; rep < 3; rep++) {
      for (int v = 0; v < 2; v++) {
        CHK(hipEventRecord(a));
        if (v == 0) hipLaunchKernelGGL((k_chain_occ<F, 0>), dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
        else hipLaunchKernelGGL((k_chain_occ<F, 3>), dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms; CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < bst[v]) bst[v] = ms;
      }
    }
    printf("  %-6s occupancy %d wave(s)/SIMD: fips %8.2f  ilp2 %8.2f G mul/s\n", name, wps,
           (double)n * ITERS / bst[0] / 1e6, (double)n * ITERS / bst[1] / 1e6);
  }
  CHK(hipFree(dx)); CHK(hipFree(dy)); CHK(hipFree(d0)); CHK(hipFree(d1));
}

int main() {
  void* h = dlopen("oracle/build/liboracle.so", RTLD_NOW);
  orc_fmul_t orc = h ? (orc_fmul_t)dlsym(h, "orc_fmul") : nullptr;
  if (!orc) printf("(oracle not loaded: %s)\n", dlerror());
  bench<FrBLS>("Fr", 0, orc);
  bench<FqBLS>("Fq", 1, orc);
  bench<FrBN>("FrBN", 2, orc);
  bench<FqBN>("FqBN", 3, orc);
  return 0;
}
