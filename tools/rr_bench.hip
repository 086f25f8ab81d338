// Reduced-radix Montgomery product (fieldrr.hpp) vs the 32-bit-limb product
// (field.hpp): correctness through the radix change, and throughput of a
// dependent chain per thread (tools only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o rr_bench rr_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../0g-ec-gpu_amd/csrc/fieldrr.hpp"

using namespace ecg;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int ITERS = 256;
constexpr int CH = 2;

template <class P>
__global__ void k_std(const Fp<P>* x, const Fp<P>* y, Fp<P>* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  Fp<P> a[CH], b = load(&y[t]);
  for (int k = 0; k < CH; k++) a[k] = load(&x[(t + k) % n]);
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int k = 0; k < CH; k++) a[k] = fmul_lz(a[k], b);
  store(&out[t], fadd(a[0], a[1]));
}

template <class Q, int SQ>
__global__ void k_rr(const Fp<typename Q::Base>* x, const Fp<typename Q::Base>* y, Fp<typename Q::Base>* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  FpR<Q> a[CH], b = rr_from_std<Q>(load(&y[t]));
  for (int k = 0; k < CH; k++) a[k] = rr_from_std<Q>(load(&x[(t + k) % n]));
  for (int i = 0; i < ITERS; i++)
    if (SQ == 2) rr_mul2(a[0], b, a[1], b, a[0], a[1]);
    else if (SQ == 3) rr_sqr2(a[0], a[1], a[0], a[1]);
    else
#pragma unroll
    for (int k = 0; k < CH; k++) a[k] = SQ ? rr_sqr(a[k]) : rr_mul(a[k], b);
  store(&out[t], rr_to_std(rr_add(a[0], a[1])));
}

// correctness: mul, sqr, add, sub, neg through the radix change vs field.hpp
template <class Q>
__global__ void k_check(const Fp<typename Q::Base>* x, const Fp<typename Q::Base>* y, uint32_t* bad, int n) {
  using F = Fp<typename Q::Base>;
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  F a = load(&x[t]), b = load(&y[t]);
  FpR<Q> ra = rr_from_std<Q>(a), rb = rr_from_std<Q>(b);
  uint32_t e = 0;
  e |= !feq(rr_to_std(rr_mul(ra, rb)), fmul(a, b)) ? 1u : 0u;
  e |= !feq(rr_to_std(rr_sqr(ra)), fmul(a, a)) ? 2u : 0u;
  e |= !feq(rr_to_std(rr_add(ra, rb)), fadd(a, b)) ? 4u : 0u;
  {
    FpR<Q> u, w;
    rr_mul2(ra, rb, rb, rb, u, w);
    e |= !feq(rr_to_std(u), fmul(a, b)) || !feq(rr_to_std(w), fmul(b, b)) ? 128u : 0u;
    rr_sqr2(ra, rb, u, w);
    e |= !feq(rr_to_std(u), fmul(a, a)) || !feq(rr_to_std(w), fmul(b, b)) ? 256u : 0u;
  }
  e |= !feq(rr_to_std(rr_sub<4>(ra, rb)), fsub(a, b)) ? 8u : 0u;
  e |= !feq(rr_to_std(rr_mul_sum2(ra, rb, rb, rr_neg<4>(ra))), fsub(fmul(a, b), fmul(b, a))) ? 512u : 0u;
  e |= !feq(rr_to_std(rr_mul_sum2(ra, rb, ra, ra)), fadd(fmul(a, b), fmul(a, a))) ? 1024u : 0u;
  e |= !feq(rr_to_std(rr_sub3<16>(ra, rb, rb, ra)), fsub(fsub(fsub(a, b), b), a)) ? 2048u : 0u;
  e |= !feq(rr_to_std(rr_mul(rr_neg_wide<4>(ra), rr_mul(rb, rb))), fmul(fneg(a), fmul(b, b))) ? 4096u : 0u;
  e |= !feq(rr_to_std(rr_neg<4>(ra)), fneg(a)) ? 16u : 0u;
  // a lazy chain: (a - b + 64p-ish) squared and multiplied stays congruent
  FpR<Q> big = rr_sub<32>(rr_sub<32>(ra, rb), rb);
  e |= !feq(rr_to_std(rr_mul(big, big)), fmul(fsub(fsub(a, b), b), fsub(fsub(a, b), b))) ? 32u : 0u;
  e |= !feq(rr_to_std(big), fsub(fsub(a, b), b)) ? 64u : 0u;
  if (e) atomicOr(bad, e);
}

static uint64_t rng_state = 0x9876543;
static uint64_t rnd() {
  rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17;
  return rng_state;
}

template <class Q>
static void run(const char* name) {
  using F = Fp<typename Q::Base>;
  const int n = 256 * 256 * 8;
  std::vector<F> hx(n), hy(n);
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < F::L; k++) { hx[i].v[k] = (uint32_t)rnd(); hy[i].v[k] = (uint32_t)rnd(); }
    hx[i].v[F::L - 1] &= 0x0fffffff; hy[i].v[F::L - 1] &= 0x0fffffff;
  }
  for (int k = 0; k < F::L; k++) { hx[0].v[k] = 0; hx[1].v[k] = F::p32(k); hy[1].v[k] = F::p32(k); }
  hx[1].v[0] -= 1; hy[1].v[0] -= 1;
  F *dx, *dy, *d0;
  uint32_t* dbad;
  CHK(hipMalloc(&dx, n * sizeof(F))); CHK(hipMalloc(&dy, n * sizeof(F))); CHK(hipMalloc(&d0, n * sizeof(F)));
  CHK(hipMalloc(&dbad, 4)); CHK(hipMemset(dbad, 0, 4));
  CHK(hipMemcpy(dx, hx.data(), n * sizeof(F), hipMemcpyHostToDevice));
  CHK(hipMemcpy(dy, hy.data(), n * sizeof(F), hipMemcpyHostToDevice));
  k_check<Q><<<n / 256, 256>>>(dx, dy, dbad, n);
  uint32_t bad = 0;
  CHK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("%s (%d x %d bits) correctness: %s (mask 0x%x)\n", name, Q::NL, Q::BITS, bad ? "FAIL" : "ok", bad);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  for (int occ : {0, 2}) {  // 0: as many waves as registers allow; 2: 2 waves/SIMD (LDS-limited)
  const size_t lds = occ ? (160 * 1024) / occ - 1024 : 0;
  printf("  occupancy: %s\n", occ ? "2 waves/SIMD" : "register-limited");
  float best[5] = {1e30f, 1e30f, 1e30f, 1e30f, 1e30f};
  for (int rep = 0; rep < 5; rep++) {
    for (int v = 0; v < 5; v++) {
      CHK(hipEventRecord(a));
      if (v == 0) hipLaunchKernelGGL(k_std<typename Q::Base>, dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
      else if (v == 1) hipLaunchKernelGGL((k_rr<Q, 0>), dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
      else if (v == 2) hipLaunchKernelGGL((k_rr<Q, 1>), dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
      else if (v == 3) hipLaunchKernelGGL((k_rr<Q, 2>), dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
      else hipLaunchKernelGGL((k_rr<Q, 3>), dim3(n / 256), dim3(256), lds, 0, dx, dy, d0, n);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms; CHK(hipEventElapsedTime(&ms, a, b));
      if (ms < best[v]) best[v] = ms;
    }
  }
  const double muls = (double)n * ITERS * CH;
  printf("  %-8s 32-bit lazy mul : %8.3f ms %8.2f G/s\n", name, best[0], muls / best[0] / 1e6);
  printf("  %-8s reduced-radix mul: %8.3f ms %8.2f G/s\n", name, best[1], muls / best[1] / 1e6);
  printf("  %-8s reduced-radix sqr: %8.3f ms %8.2f G/s\n", name, best[2], muls / best[2] / 1e6);
  printf("  %-8s rr paired mul    : %8.3f ms %8.2f G/s\n", name, best[3], muls / best[3] / 1e6);
  printf("  %-8s rr paired sqr    : %8.3f ms %8.2f G/s\n", name, best[4], muls / best[4] / 1e6);
  }
  CHK(hipFree(dx)); CHK(hipFree(dy)); CHK(hipFree(d0)); CHK(hipFree(dbad));
}

int main() {
  run<params::bls12_381_fq_rr>("BLS-Fq");
  run<params::bn254_fq_rr>("BN-Fq");
  return 0;
}
