// Lane-shared point adds against the single-lane formulas (tools only): for
// G1 (BLS12-381 13 x 30) and G2 (BLS12-381 Fq2, 14 x 29), random XYZZ
// coordinates p, q and the exceptional operands q = p (doubling branch) and
// q = -p (identity branch), every lane group's pp_add / pp_dbl result is
// compared with rr_add_xyzz / r2_add_xyzz and rr_dbl / r2_dbl limb for limb
// and as a point (cross-multiplied coordinates, canonical).
// Build: hipcc --offload-arch=gfx950 -O3 -I../0g-ec-gpu_amd/csrc -o lane_add_check lane_add_check.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "curve_rr2.hpp"

using namespace ecg;

// random field elements below p: limbs < 2^28, the top limb < 8 (value < 2^380)
template <class Q>
__device__ void rand_fill(FpR<Q>& a, uint64_t seed) {
  for (int i = 0; i < Q::NL; i++) {
    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
    a.v[i] = (uint32_t)(seed >> 40) & ((1u << 28) - 1);
  }
  a.v[Q::NL - 1] &= 7u;
}
template <class Q>
__device__ void rand_fill(FpR2<Q>& a, uint64_t seed) {
  rand_fill(a.c0, seed);
  rand_fill(a.c1, seed ^ 0x9E3779B97F4A7C15ull);
}

template <class Q>
__device__ FpR<Q> pa_mul(const FpR<Q>& a, const FpR<Q>& b) { return rr_mul(a, b); }
template <class Q>
__device__ FpR2<Q> pa_mul(const FpR2<Q>& a, const FpR2<Q>& b) { return r2_mul<4>(a, b); }
template <class Q>
__device__ bool canon_eq(const FpR<Q>& a, const FpR<Q>& b) {
  const auto x = rr_to_std(a), y = rr_to_std(b);
  bool e = true;
  for (int i = 0; i < decltype(x)::L; i++) e = e && x.v[i] == y.v[i];
  return e;
}
template <class Q>
__device__ bool canon_eq(const FpR2<Q>& a, const FpR2<Q>& b) { return canon_eq(a.c0, b.c0) && canon_eq(a.c1, b.c1); }

// mode 0: p + q random; 1: p + p; 2: p + (-p) (Y negated: kp - Y); 3: 2p
template <class F, int PM>
__global__ void check_kernel(int mode, uint32_t* bad) {
  constexpr uint32_t LB = pp_lanes_log<PM>();
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t id = gid >> LB;
  XYZZ<F> p, q;
  rand_fill(p.X, id * 4 + 1);
  rand_fill(p.Y, id * 4 + 2);
  rand_fill(p.ZZ, id * 4 + 3);
  rand_fill(p.ZZZ, id * 4 + 4);
  q = p;
  if (mode == 0) {
    rand_fill(q.X, id * 4 + 1001);
    rand_fill(q.Y, id * 4 + 1002);
  }
  if (mode == 2) q.Y = pa_neg_y(p.Y);
  XYZZ<F> want, got;
  if (mode == 3) {
    want = pa_dbl(p);
    got = pp_dbl<PM>(p);
  } else {
    want = pa_add(p, q);
    got = pp_add<PM>(p, q);
  }
  const uint32_t* a = reinterpret_cast<const uint32_t*>(&want);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(&got);
  uint32_t diff = 0;
  for (size_t i = 0; i < sizeof(want) / 4; i++) diff |= a[i] ^ b[i];
  if (diff) atomicAdd(&bad[0], 1u);
  // the same point: X1 ZZ2 = X2 ZZ1, Y1 ZZZ2 = Y2 ZZZ1 (mod p), both identity, or neither
  const bool wz = pa_is_zero(want), gz = pa_is_zero(got);
  bool same = wz == gz;
  if (same && !wz) same = canon_eq(pa_mul(want.X, got.ZZ), pa_mul(got.X, want.ZZ)) &&
                          canon_eq(pa_mul(want.Y, got.ZZZ), pa_mul(got.Y, want.ZZZ));
  if (!same) atomicAdd(&bad[1], 1u);
}

template <class F, int PM>
static int run(const char* name) {
  uint32_t* bad;
  if (hipMalloc(&bad, 8) != hipSuccess) return 1;
  for (int mode = 0; mode < 4; mode++) {
    if (hipMemset(bad, 0, 8) != hipSuccess) return 1;
    hipLaunchKernelGGL((check_kernel<F, PM>), dim3(64), dim3(256), 0, 0, mode, bad);
    uint32_t h[2] = {0, 0};
    if (hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("%-4s PM=%d mode %d (%s): limbs differ on %u, points differ on %u of %u lanes\n", name, PM, mode,
           mode == 0 ? "p+q" : mode == 1 ? "p+p" : mode == 2 ? "p-p" : "2p", h[0], h[1], 64u * 256u);
  }
  hipFree(bad);
  return 0;
}

int main() {
  using G1 = FpR<params::bls12_381_fq13_rr>;
  using G2 = FpR2<params::bls12_381_fq_rr>;
  int rc = 0;
  rc |= run<G1, 1>("G1");
  rc |= run<G1, 4>("G1");
  rc |= run<G2, 1>("G2");
  rc |= run<G2, 4>("G2");
  return rc;
}
