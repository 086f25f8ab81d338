// Batch-affine accumulation costed on the device: the
// cost of one affine point addition whose inversion is shared by a batch
// (Montgomery's trick), against the XYZZ mixed add the accumulation runs
// (curve_rr.hpp rr_add_affine, madd-2008-s), both in the 13 x 30-bit
// reduced-radix BLS12-381 Fq of the product path.
//
//   xyzz          : each lane runs a dependent chain of mixed adds, as
//                   msm_accumulate_kernel does (acc += P_i).
//   affine<K,WG>  : each lane adds K independent point pairs (A_k + B_k ->
//                   C_k, all affine): prefix products c_k of dx_k, ONE
//                   inversion, back-substitution (inv_k = inv c_{k-1},
//                   inv *= dx_k), then lambda = dy inv_k, x3 = lambda^2 - xA -
//                   xB, y3 = lambda (xA - x3) - yA.  5M + 1S per add plus the
//                   inversion's share.  WG = 0: one Fermat inversion per lane;
//                   WG = 1: the lanes' products meet in an LDS product tree
//                   (256 lanes), one lane inverts the root, the tree hands
//                   each lane the inverse of its own product.  K <= 8 keeps
//                   the prefix products in registers; K > 8 parks them in
//                   global scratch (what a whole-segment batch needs).
// Every variant checks its first lanes' results against rr_add_affine
// (x3 ZZ == X, y3 ZZZ == Y, canonical) and folds all results into a
// checksum, so nothing is dead code.  Bases: 4096 affine points (x, y as
// 12-u64 Montgomery records) read from the file given as argv[1]
// (tools/batch_affine_bench.py writes it from the CPU oracle).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o batch_affine_bench batch_affine_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../0g-ec-gpu_amd/csrc/curve_rr.hpp"

using namespace ecg;
using Q = params::bls12_381_fq13_rr;
using F = FpR<Q>;
using SF = Fp<Q::Base>;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int TB = 4096;       // table of bases (L2-resident, as hot records would be)
constexpr int THREADS = 256;

// p - 2 of BLS12-381 Fq, little-endian u64 words
__constant__ uint64_t PM2[6] = {0xb9feffffffffaaa9ull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                                0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};

ECG_DEV F rr_inv(const F& a) {  // a^(p-2), square-and-multiply from the top bit (uniform branches)
  F r = a;  // bit 380, the top bit of p - 2
  for (int b = 379; b >= 0; b--) {
    r = rr_sqr(r);
    if ((PM2[b >> 6] >> (b & 63)) & 1) r = rr_mul(r, a);
  }
  return r;
}

ECG_DEV Affine<F> base(const Affine<F>* tab, uint32_t i) { return tab[i & (TB - 1)]; }

ECG_DEV void fold(uint32_t& sum, const F& v) {
#pragma unroll
  for (int i = 0; i < Q::NL; i++) sum ^= v.v[i] * (2 * i + 1);
}

__global__ void k_to_rr(const SF* xy, Affine<F>* tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TB) return;
  tab[i].x = rr_reduce_q(rr_from_std<Q>(load(&xy[2 * i])));
  tab[i].y = rr_reduce_q(rr_from_std<Q>(load(&xy[2 * i + 1])));
}

// the accumulation's own chain: acc += P_i, `adds` per lane
__global__ void __launch_bounds__(THREADS) k_xyzz(const Affine<F>* tab, int adds, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  XYZZ<F> acc = xyzz_zero<F>();
  for (int i = 0; i < adds; i++) acc = rr_add_affine(acc, base(tab, t * 7 + i * 13));
  uint32_t s = 0;
  fold(s, acc.X);
  fold(s, acc.ZZ);
  out[t] = s;
}

// one affine add C = A + B given inv = 1 / (xB - xA)
ECG_DEV void aff_finish(const Affine<F>& A, const Affine<F>& B, const F& inv, F& x3, F& y3) {
  const F lam = rr_mul(rr_sub<4>(B.y, A.y), inv);
  x3 = rr_reduce_q(rr_sub2<8>(rr_sqr(lam), A.x, B.x));
  y3 = rr_reduce_q(rr_sub<4>(rr_mul(lam, rr_sub<4>(A.x, x3)), A.y));
}

// LDS product tree over the workgroup's lanes: in = this lane's product,
// returns the inverse of it (one inversion per workgroup)
ECG_DEV F wg_invert(const F& in, uint32_t* lds) {
  constexpr int NW = Q::NL;
  auto put = [&](int node, const F& v) {
#pragma unroll
    for (int i = 0; i < NW; i++) lds[i * 2 * THREADS + node] = v.v[i];
  };
  auto get = [&](int node) {
    F v;
#pragma unroll
    for (int i = 0; i < NW; i++) v.v[i] = lds[i * 2 * THREADS + node];
    return v;
  };
  uint32_t* inv_lds = lds + NW * 2 * THREADS;
  auto iput = [&](int node, const F& v) {
#pragma unroll
    for (int i = 0; i < NW; i++) inv_lds[i * 2 * THREADS + node] = v.v[i];
  };
  auto iget = [&](int node) {
    F v;
#pragma unroll
    for (int i = 0; i < NW; i++) v.v[i] = inv_lds[i * 2 * THREADS + node];
    return v;
  };
  const int t = threadIdx.x;
  put(THREADS + t, in);
  __syncthreads();
  for (int cnt = THREADS / 2; cnt >= 1; cnt >>= 1) {  // nodes [cnt, 2 cnt)
    if (t < cnt) put(cnt + t, rr_mul(get(2 * (cnt + t)), get(2 * (cnt + t) + 1)));
    __syncthreads();
  }
  if (t == 0) iput(1, rr_inv(get(1)));
  __syncthreads();
  for (int cnt = 1; cnt < THREADS; cnt <<= 1) {  // children of nodes [cnt, 2 cnt)
    if (t < cnt) {
      const int nd = cnt + t;
      const F iv = iget(nd);
      F l, r;
      rr_mul2(iv, get(2 * nd + 1), iv, get(2 * nd), l, r);
      iput(2 * nd, l);
      iput(2 * nd + 1, r);
    }
    __syncthreads();
  }
  return iget(THREADS + t);
}

template <int K, bool WG>
__global__ void __launch_bounds__(THREADS) k_affine(const Affine<F>* tab, int rounds, uint32_t* scratch,
                                                    uint32_t* out, uint32_t* bad) {
  __shared__ uint32_t lds[WG ? 2 * Q::NL * 2 * THREADS : 1];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nl = gridDim.x * blockDim.x;
  uint32_t s = 0;
  constexpr bool REG = K <= 8;
  F creg[REG ? K : 1];
  for (int rd = 0; rd < rounds; rd++) {
    const uint32_t i0 = t * 7 + rd * 4099 * K;
    // prefix products of dx_k
    F c = F::one();
#pragma unroll(REG ? K : 4)
    for (int k = 0; k < K; k++) {
      const Affine<F> A = base(tab, i0 + 2 * k), B = base(tab, i0 + 2 * k + 1);
      c = rr_mul(c, rr_sub<4>(B.x, A.x));
      if constexpr (REG) {
        creg[k] = c;
      } else {
#pragma unroll
        for (int i = 0; i < Q::NL; i++) scratch[((size_t)k * Q::NL + i) * nl + t] = c.v[i];
      }
    }
    F inv;
    if constexpr (WG)
      inv = wg_invert(c, lds);
    else
      inv = rr_inv(c);
    // back-substitution, last pair first
#pragma unroll(REG ? K : 4)
    for (int k = K - 1; k >= 0; k--) {
      const Affine<F> A = base(tab, i0 + 2 * k), B = base(tab, i0 + 2 * k + 1);
      F inv_k;
      if (k == 0) {
        inv_k = inv;
      } else {
        F cp;
        if constexpr (REG) {
          cp = creg[k - 1];
        } else {
#pragma unroll
          for (int i = 0; i < Q::NL; i++) cp.v[i] = scratch[((size_t)(k - 1) * Q::NL + i) * nl + t];
        }
        F ni;
        rr_mul2(inv, cp, inv, rr_sub<4>(B.x, A.x), inv_k, ni);
        inv = ni;
      }
      F x3, y3;
      aff_finish(A, B, inv_k, x3, y3);
      fold(s, x3);
      fold(s, y3);
      if (rd == 0 && t < 64) {  // check against the XYZZ mixed add
        XYZZ<F> acc;
        acc.X = A.x;
        acc.Y = A.y;
        acc.ZZ = F::one();
        acc.ZZZ = F::one();
        acc = rr_add_affine(acc, B);
        const bool okx = feq(rr_to_std(rr_mul(x3, acc.ZZ)), rr_to_std(acc.X));
        const bool oky = feq(rr_to_std(rr_mul(y3, acc.ZZZ)), rr_to_std(acc.Y));
        if (!okx || !oky) atomicAdd(bad, 1u);
      }
    }
  }
  out[t] = s;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <bases.bin: 4096 x 12 u64>\n", argv[0]);
    return 2;
  }
  std::vector<uint64_t> h(TB * 12);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(h.data(), 8, h.size(), f) != h.size()) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  SF* d_xy;
  Affine<F>* tab;
  CHK(hipMalloc(&d_xy, h.size() * 8));
  CHK(hipMalloc(&tab, TB * sizeof(Affine<F>)));
  CHK(hipMemcpy(d_xy, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_to_rr, dim3(TB / 256), dim3(256), 0, 0, d_xy, tab);
  const int blocks = 256 * 8;  // 8 workgroups per CU
  const size_t lanes = (size_t)blocks * THREADS;
  uint32_t *out, *bad, *scratch;
  CHK(hipMalloc(&out, lanes * 4));
  CHK(hipMalloc(&bad, 4));
  CHK(hipMalloc(&scratch, lanes * 1024 * Q::NL * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto time = [&](const char* name, double adds_per_lane, auto launch) {
    CHK(hipMemset(bad, 0, 4));
    launch();  // warm
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      CHK(hipEventRecord(e0));
      launch();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    uint32_t nb = 0;
    CHK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
    const double adds = adds_per_lane * lanes;
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"adds\": %.0f, \"ns_per_add_per_cu\": %.2f, \"adds_per_s\": %.4g, "
           "\"check_failures\": %u}\n",
           name, best, adds, best * 1e6 / adds * 256, adds / (best * 1e-3), nb);
    fflush(stdout);
  };
  const int ADDS = 256;
  time("xyzz_madd_chain", ADDS, [&] { hipLaunchKernelGGL(k_xyzz, dim3(blocks), dim3(THREADS), 0, 0, tab, ADDS, out); });
#define AFF(K, WG, R)                                                                                   \
  time(WG ? "affine_K" #K "_wg" : "affine_K" #K "_lane", (double)(K) * (R), [&] {                      \
    hipLaunchKernelGGL((k_affine<K, WG>), dim3(blocks), dim3(THREADS), 0, 0, tab, R, scratch, out, bad); \
  });
  AFF(1, false, 8)
  AFF(8, false, 8)
  AFF(64, false, 2)
  AFF(1, true, 16)
  AFF(4, true, 16)
  AFF(8, true, 8)
  AFF(16, true, 8)
  AFF(64, true, 2)
  AFF(256, false, 1)
  AFF(1024, false, 1)
  CHK(hipGetLastError());
  return 0;
}
