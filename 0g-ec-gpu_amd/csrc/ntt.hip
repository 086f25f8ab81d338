// Radix-2^DEG Stockham NTT over the scalar fields (BLS12-381 Fr, BN254 Fr).
//
// Replaces FIELD_radix_fft (ag-build/cl/fft.cl:4-68) and its host driver
// SingleFftKernel::radix_fft (ec-gpu-proxy/src/fft.rs:50-135).  Same
// decomposition (Stockham autosort: natural order in and out, each pass a
// batch of independent 2^deg-point DFTs between a strided gather and a
// scatter), re-designed for gfx950:
//
//  * v2 (default): ceil(log n / 10) balanced passes of radix up to 2^10
//    (2^24 is three passes of 2^8; ECG_NTT_MAXDEG up to 12 for A/B).  A
//    pass's groups are packed into 1024-element tiles in LDS worked by
//    256-thread workgroups, so every global read is a G*32-byte run.  Each
//    thread runs TWO DIF rounds per LDS round trip on 4 register-resident
//    elements (radix-2^2 step), halving LDS traffic and barriers.
//  * The butterflies run in the reduced-radix form (ntt_pass_rr_kernel, see
//    its header) whenever the full per-pass twiddle tables fit (log n <= 28):
//    ~1/3 fewer VALU instructions per product.  ECG_NTT_RR=0 keeps the
//    32-bit-limb passes below for A/B.
//  * No per-thread exponentiation (the reference's FIELD_pow_lookup + FIELD_pow
//    per thread, fft.cl:39-45, ~4x the butterfly work): inter-pass twiddles
//    w^e (e < n) = T_hi[e >> 12] * T_lo[e & 4095] from L2-resident tables;
//    in-group roots from a 2^(maxdeg-1) table.  Tables are built on the device
//    once per (omega, log n) and cached in the context.
//  * Values stay fully reduced (< r): output bytes equal serial_fft's.
//  * v1 (ECG_NTT_VARIANT=1): radix-2^8 passes, one DIF round per LDS round
//    trip -- kept for A/B measurement.
#include <cstdlib>
#include <cstring>

#include "ctx.hpp"
#include "field.hpp"
#include "fieldrr.hpp"

namespace ecg {

constexpr int NTT_LO_BITS = 12;  // twiddle split table size 2^12

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

// twiddle w^e for e < n from the split tables
template <class F>
ECG_DEV F twiddle(const F* __restrict__ tw_lo, const F* __restrict__ tw_hi, uint64_t e) {
  return fmul(load(&tw_hi[e >> NTT_LO_BITS]), load(&tw_lo[e & ((1u << NTT_LO_BITS) - 1)]));
}

// ---------------------------------------------------------------------------
// shared load / store phases of a Stockham pass
//   u[i] = x[g + i*t] * w^((n >> (lgp+DEG)) * k * i),  k = g mod 2^lgp, t = n >> DEG
//   y[(g - k)*2^DEG + k + j*2^lgp] = v[j]   (v = DFT of u, natural order)
// ---------------------------------------------------------------------------
// A thread owns at most NTT_EPT elements of the tile (launch: threads >= E /
// NTT_EPT).  Every global load of the tile -- elements and twiddles -- is
// issued before the first product, so a tile waits for one HBM latency, not
// one per element (the strided loop over a runtime bound could not unroll).
constexpr int NTT_EPT = 4;

template <class F, int DEG>
ECG_DEV void pass_load(const F* __restrict__ x, const F* __restrict__ tw_lo, const F* __restrict__ tw_hi,
                       const F* __restrict__ twf, const LdsPlanes<F>& U, uint32_t log_n, uint32_t lgp,
                       uint32_t log_g, uint32_t E) {
  const uint32_t G = 1u << log_g;
  const uint64_t t = (1ull << log_n) >> DEG;
  const uint64_t p = 1ull << lgp;
  const uint64_t g0 = (uint64_t)blockIdx.x << log_g;
  const uint32_t s_tw_log = log_n - lgp - DEG;  // n >> (lgp + DEG) = 2^s_tw_log
  F v[NTT_EPT], w[NTT_EPT];
  bool mul[NTT_EPT];
#pragma unroll
  for (int q = 0; q < NTT_EPT; q++) {
    const uint32_t f = threadIdx.x + q * blockDim.x;
    mul[q] = false;
    if (f < E) {
      const uint32_t gi = f & (G - 1), i = f >> log_g;
      const uint64_t g = g0 + gi;
      v[q] = load(&x[g + (uint64_t)i * t]);
      if (lgp != 0) {
        const uint64_t k = g & (p - 1);
        const uint64_t e = (k * i) << s_tw_log;  // < n
        if (e != 0) {
          // full per-pass table twf[i * p + k] (one load, k contiguous across
          // lanes) or the split tables (two loads + one product)
          mul[q] = true;
          w[q] = twf ? load(&twf[(uint64_t)i * p + k]) : twiddle(tw_lo, tw_hi, e);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NTT_EPT; q++) {
    const uint32_t f = threadIdx.x + q * blockDim.x;
    if (f < E) {
      if (mul[q]) v[q] = fmul(v[q], w[q]);
      U.put(((f & (G - 1)) << DEG) + (f >> log_g), v[q]);
    }
  }
}

template <class F, int DEG>
ECG_DEV void pass_store(F* __restrict__ y, const LdsPlanes<F>& U, uint32_t lgp, uint32_t log_g, uint32_t E) {
  constexpr uint32_t R = 1u << DEG;
  const uint64_t p = 1ull << lgp;
  const uint64_t g0 = (uint64_t)blockIdx.x << log_g;
  const uint32_t lpp = lgp < log_g ? lgp : log_g;  // lanes walk min(p, G) fastest -> contiguous runs
  const uint32_t pp = 1u << lpp;
#pragma unroll
  for (int q = 0; q < NTT_EPT; q++) {
    const uint32_t f = threadIdx.x + q * blockDim.x;
    if (f >= E) break;
    const uint32_t kk = f & (pp - 1);
    const uint32_t j = (f >> lpp) & (R - 1);
    const uint32_t gh = f >> (lpp + DEG);
    const uint32_t gi = (gh << lpp) + kk;
    const uint64_t g = g0 + gi;
    const uint64_t k = g & (p - 1);
    store(&y[((g - k) << DEG) + k + (uint64_t)j * p], U.get((gi << DEG) + bitrev(j, DEG)));
  }
}

// ---------------------------------------------------------------------------
// v2 pass: DEG <= 12, two DIF rounds per LDS round trip
// ---------------------------------------------------------------------------
// threads per workgroup = max(2^DEG, 1024) / 4 (see launch_pass)
template <class P, int DEG>
__global__ void __launch_bounds__(1024)
    ntt_pass_kernel(const Fp<P>* __restrict__ x, Fp<P>* __restrict__ y, const Fp<P>* __restrict__ pq,
                    uint32_t pq_shift, const Fp<P>* __restrict__ tw_lo, const Fp<P>* __restrict__ tw_hi,
                    const Fp<P>* __restrict__ twf, uint32_t log_n, uint32_t lgp, uint32_t log_g) {
  using F = Fp<P>;
  static_assert(F::L == 8, "NTT tiles assume 32-byte scalar-field elements");
  constexpr uint32_t R = 1u << DEG;
  extern __shared__ uint4 smem[];
  const uint32_t E = R << log_g;
  LdsPlanes<F> U{smem, smem + E};

  pass_load<F, DEG>(x, tw_lo, tw_hi, twf, U, log_n, lgp, log_g, E);
  __syncthreads();

  // radix-2^2 steps: rounds r and r+1 of the DIF network on quartets
  // {j, j+h, j+2h, j+3h} (h = bit/2, bit = R/2 >> r); root w = w_{2^DEG}.
  int r = 0;
  constexpr uint32_t RQ = R >= 4 ? R / 4 : 1;  // quartets per group
#pragma unroll 1
  for (; r + 1 < DEG; r += 2) {
    const uint32_t bit = (R / 2) >> r, h = bit >> 1;
    for (uint32_t f = threadIdx.x; f < E / 4; f += blockDim.x) {
      const uint32_t gi = f / RQ, q = f % RQ;
      const uint32_t qm = q & (h - 1);
      const uint32_t j = (gi << DEG) + ((q / h) * (2 * bit)) + qm;
      F e0 = U.get(j), e1 = U.get(j + h), e2 = U.get(j + bit), e3 = U.get(j + bit + h);
      // round r: (e0, e2) twiddle w^(qm << r), (e1, e3) twiddle w^((qm + h) << r)
      F s0 = fadd(e0, e2), d0 = fsub(e0, e2);
      F s1 = fadd(e1, e3), d1 = fsub(e1, e3);
      if (qm != 0) d0 = fmul(d0, load(&pq[(uint64_t)(qm << r) << pq_shift]));
      d1 = fmul(d1, load(&pq[(uint64_t)((qm + h) << r) << pq_shift]));
      // round r+1: pairs (s0, s1) and (d0, d1), both twiddle w^(qm << (r+1))
      F a0 = fadd(s0, s1), a1 = fsub(s0, s1);
      F b0 = fadd(d0, d1), b1 = fsub(d0, d1);
      if (qm != 0) {
        const F w2 = load(&pq[(uint64_t)(qm << (r + 1)) << pq_shift]);
        a1 = fmul(a1, w2);
        b1 = fmul(b1, w2);
      }
      U.put(j, a0);
      U.put(j + h, a1);
      U.put(j + bit, b0);
      U.put(j + bit + h, b1);
    }
    __syncthreads();
  }
  if (r < DEG) {  // odd DEG: last radix-2 round (bit = 1, all twiddles trivial)
    for (uint32_t f = threadIdx.x; f < E / 2; f += blockDim.x) {
      const uint32_t i0 = 2 * f;
      F u0 = U.get(i0), u1 = U.get(i0 + 1);
      U.put(i0, fadd(u0, u1));
      U.put(i0 + 1, fsub(u0, u1));
    }
    __syncthreads();
  }
  pass_store<F, DEG>(y, U, lgp, log_g, E);
}

// ---------------------------------------------------------------------------
// v1 pass (A/B): radix-2^8, one radix-2 round per LDS round trip, 256 threads
// ---------------------------------------------------------------------------
template <class P, int DEG>
__global__ void __launch_bounds__(256)
    ntt_pass_v1_kernel(const Fp<P>* __restrict__ x, Fp<P>* __restrict__ y, const Fp<P>* __restrict__ pq,
                       uint32_t pq_shift, const Fp<P>* __restrict__ tw_lo, const Fp<P>* __restrict__ tw_hi,
                       const Fp<P>* __restrict__ twf, uint32_t log_n, uint32_t lgp, uint32_t log_g) {
  using F = Fp<P>;
  constexpr uint32_t R = 1u << DEG;
  extern __shared__ uint4 smem[];
  const uint32_t E = R << log_g;
  LdsPlanes<F> U{smem, smem + E};
  pass_load<F, DEG>(x, tw_lo, tw_hi, twf, U, log_n, lgp, log_g, E);
  __syncthreads();
#pragma unroll 1
  for (int rnd = 0; rnd < DEG; rnd++) {
    const uint32_t bit = (R / 2) >> rnd;
    for (uint32_t f = threadIdx.x; f < E / 2; f += blockDim.x) {
      const uint32_t gi = f >> (DEG - 1), b = f & (R / 2 - 1);
      const uint32_t di = b & (bit - 1);
      const uint32_t i0 = (gi << DEG) + (b << 1) - di, i1 = i0 + bit;
      F u0 = U.get(i0), u1 = U.get(i1);
      F s = fadd(u0, u1);
      F d = fsub(u0, u1);
      if (di != 0) d = fmul(d, load(&pq[(uint64_t)(di << rnd) << pq_shift]));
      U.put(i0, s);
      U.put(i1, d);
    }
    __syncthreads();
  }
  pass_store<F, DEG>(y, U, lgp, log_g, E);
}

// ---------------------------------------------------------------------------
// Reduced-radix pass (default for both scalar fields): the same Stockham
// schedule, with the butterflies in the 9 x 29-bit form of fieldrr.hpp.  An
// Fr product is then 162 v_mad_u64_u32 and no carry instructions (the 32-bit
// form above issues 128 mads + 128 addc + the final subtraction), and sums /
// differences are limb-wise with no carry chain.
//
// No conversion product anywhere: the caller's word x R (< r) is re-read as a
// 9-limb integer, i.e. as the reduced-radix form of x R / R' (R' = 2^261).
// The transform is linear, so the output integers are y R / R' * R' = y R --
// exactly the boundary form -- once packed back into 8 words.  Twiddles are
// stored in the R' form (converted once when the tables are built).
//
// Values between butterfly rounds ("E-form"): exact limbs, value <= 2.5 r.
// A radix-2^2 step on e0..e3 (r / R' <= 2^-6.1; products take one operand
// with limbs < 2^31.6 against an exact twiddle and return < r (1 + K 2^-6.1)):
//   s0 = e0 + e2, d0 = (e0 + 8r - e2) w0        (<= 5 r,  <= 1.15 r)
//   s1 = e1 + e3, d1 = (e1 + 8r - e3) w1
//   a0 = reduce_q(s0 + s1)                      (<= 1.1 r)
//   a1 = (s0 + 16r - s1) w2                     (<= 1.3 r)
//   b0 = carry(d0 + d1)                         (<= 2.3 r)
//   b1 = (d0 + 4r - d1) w2                      (<= 1.1 r)
// The last step of a pass (h = 1: three of its four twiddles are 1, or the
// radix-2 round of an odd DEG) leaves its outputs unreduced ("P-form": limbs
// < 2^31.4, value <= 21 r): they meet a product next -- the following pass
// multiplies every element by its twiddle first, and a product of such an
// operand with an exact twiddle is < r (1 + 21 * 2^-6.1) < 1.4 r with exact
// limbs (column sums < 9 2^60.4 + 9 2^58 < 2^64) -- or rr_store_std's
// reduce_q (limbs < 2^31.4, value < 64 r).  The first pass reads canonical
// input and has no twiddle product, so P-form values never enter a sum.
//
// HBM layout: the transform's input and output are the boundary layout
// (canonical, 8 packed words).  Between passes the elements stay in the
// P-form as three planes (limbs 0-3 | 4-7 | 8: 36 B per element, coalesced
// 16-B / 4-B accesses), so an inner pass boundary costs no unpacking,
// reduction, canonicalisation or packing (~125 VALU instructions per element
// saved for 4 more bytes).  The twiddle tables are planes of exact canonical
// limbs for the same reason.
// ---------------------------------------------------------------------------
template <class Q>
struct RrPlanes {  // limbs 0-3 | 4-7 | 8 of element i (NL = 9)
  uint4* a;
  uint4* b;
  uint32_t* c;
  ECG_HD static RrPlanes over(void* base, size_t n) {
    uint4* p = reinterpret_cast<uint4*>(base);
    return RrPlanes{p, p + n, reinterpret_cast<uint32_t*>(p + 2 * n)};
  }
  ECG_HD RrPlanes at(size_t off) const { return RrPlanes{a + off, b + off, c + off}; }
  ECG_DEV FpR<Q> get(size_t i) const {
    static_assert(Q::NL == 9, "three planes hold 9 limbs");
    const uint4 x = a[i], y = b[i];
    FpR<Q> r;
    r.v[0] = x.x; r.v[1] = x.y; r.v[2] = x.z; r.v[3] = x.w;
    r.v[4] = y.x; r.v[5] = y.y; r.v[6] = y.z; r.v[7] = y.w;
    r.v[8] = c[i];
    return r;
  }
  ECG_DEV void put(size_t i, const FpR<Q>& v) const {
    a[i] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
    b[i] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
    c[i] = v.v[8];
  }
};
constexpr size_t RR_PLANE_BYTES = 36;  // bytes per element in the plane layout

template <class Q>
ECG_DEV FpR<Q> rr_load_std(const uint4* __restrict__ x, size_t i) {  // 8 words x R -> 9 exact limbs
  const uint4 lo = x[2 * i], hi = x[2 * i + 1];
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  FpR<Q> r;
  rr_unpack<Q, 8>(w, r.v);
  return r;
}

template <class Q>
ECG_DEV void rr_store_std(uint4* __restrict__ y, size_t i, const FpR<Q>& v) {  // E-form -> canonical 8 words
  const FpR<Q> c = rr_canon_lt2p(rr_reduce_q(v));
  uint32_t w[8];
  rr_pack<Q, 8>(c.v, w);
  y[2 * i] = make_uint4(w[0], w[1], w[2], w[3]);
  y[2 * i + 1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// LDS layout: the three planes, unswizzled.  A linear XOR swizzle of the
// element slots (found by a bank simulation of every access pattern of the
// 1024-element tiles) cut SQ_LDS_BANK_CONFLICT from 1354 to 96 cycles per wave
// but left the pass time unchanged and added ~3% VALU instructions for the
// slot arithmetic: the pass is VALU-issue-bound (SQ_INSTS_VALU x 4 cycles ~
// 0.94 of the wave cycles at 4 waves/SIMD), not LDS-bound
// (profiles/r02b/ntt_lds_swizzle.txt).
ECG_HD constexpr uint32_t lds_phys(uint32_t j) { return j; }

// Up to 1024 threads (4096-element tiles, 147 KB of LDS: the 2-pass 2^24
// schedule of ECG_NTT_MAXDEG=12); 4 waves/SIMD bound the kernel to 128 VGPRs
// either way.
constexpr uint32_t NTT_RR_THREADS = 1024;

#ifndef ECG_NTT_RR_WAVES
#define ECG_NTT_RR_WAVES 4
#endif
// IN_RR / OUT_RR: the pass reads / writes the plane layout (inner pass
// boundaries) instead of the boundary layout.
template <class Q, int DEG, bool IN_RR, bool OUT_RR>
__global__ void __launch_bounds__(NTT_RR_THREADS) __attribute__((amdgpu_waves_per_eu(ECG_NTT_RR_WAVES)))
    ntt_pass_rr_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, const uint4* __restrict__ pq_base,
                       uint32_t pq_cnt, uint32_t pq_shift, const uint4* __restrict__ twf_base, uint64_t twf_cnt,
                       uint64_t twf_off, uint32_t log_n, uint32_t lgp, uint32_t log_g, uint32_t xcd_runs,
                       uint32_t log_tiles) {
  using F = FpR<Q>;
  constexpr uint32_t R = 1u << DEG;
  extern __shared__ uint4 smem[];
  const uint32_t E = R << log_g;
  const RrPlanes<Q> U = RrPlanes<Q>::over(smem, E);
  const uint32_t G = 1u << log_g;
  const size_t n = (size_t)1 << log_n;
  // XCD-aware tile order (xcd_runs): blocks b and b + 8 share an XCD (round-robin
  // dispatch), so XCD b % 8 takes a contiguous run of tiles.  Neighbouring tiles
  // share the 128-B lines of the planes (4 columns of 16 + 16 + 4 B per tile
  // row) and now meet in one L2 instead of fetching each line once per XCD.
  const uint32_t tile_all = xcd_runs ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  // batched transforms (radix_fft_many): transform tile_all >> log_tiles of the
  // batch, stored back to back in the input's and the output's layout
  const uint32_t tile = tile_all & ((1u << log_tiles) - 1);
  const size_t tix = tile_all >> log_tiles;
  x += tix * (IN_RR ? ((size_t)9 << log_n) / 4 : (size_t)2 << log_n);  // 36 B or 32 B per element, in uint4
  y += tix * (OUT_RR ? ((size_t)9 << log_n) / 4 : (size_t)2 << log_n);
  const uint64_t g0 = (uint64_t)tile << log_g;
  const RrPlanes<Q> PQ = RrPlanes<Q>::over(const_cast<uint4*>(pq_base), pq_cnt);

  // ---- load: u[i] = x[g + i t] * w^((n >> (lgp + DEG)) k i) (full per-pass table)
  {
    const uint64_t t = n >> DEG;
    const uint64_t p = 1ull << lgp;
    F v[NTT_EPT];
#pragma unroll
    for (int q = 0; q < NTT_EPT; q++) {
      const uint32_t f = threadIdx.x + q * blockDim.x;
      v[q] = F::zero();
      if (f < E) {
        const uint64_t src = g0 + (f & (G - 1)) + (uint64_t)(f >> log_g) * t;
        if constexpr (IN_RR)
          v[q] = RrPlanes<Q>::over(const_cast<uint4*>(x), n).get(src);
        else
          v[q] = rr_load_std<Q>(x, src);
      }
    }
    if (lgp != 0) {  // every element times its twiddle (w^0 = 1 is a table entry too: no divergence)
      const RrPlanes<Q> TW = RrPlanes<Q>::over(const_cast<uint4*>(twf_base), twf_cnt).at(twf_off);
      F w[NTT_EPT];
#pragma unroll
      for (int q = 0; q < NTT_EPT; q++) {
        const uint32_t f = threadIdx.x + q * blockDim.x;
        const uint64_t g = g0 + (f & (G - 1));
        w[q] = f < E ? TW.get((uint64_t)(f >> log_g) * p + (g & (p - 1))) : F::one();
      }
#pragma unroll
      for (int q = 0; q + 1 < NTT_EPT; q += 2) {
        F p0, p1;
        rr_mul2(v[q], w[q], v[q + 1], w[q + 1], p0, p1);
        v[q] = p0;
        v[q + 1] = p1;
      }
    }
#pragma unroll
    for (int q = 0; q < NTT_EPT; q++) {
      const uint32_t f = threadIdx.x + q * blockDim.x;
      if (f < E) U.put(lds_phys(((f & (G - 1)) << DEG) + (f >> log_g)), v[q]);
    }
  }
  __syncthreads();

  // ---- radix-2^2 steps (rounds r, r+1 of the DIF network)
  int r = 0;
  constexpr uint32_t RQ = R >= 4 ? R / 4 : 1;
#pragma unroll 1
  for (; r + 1 < DEG; r += 2) {
    const uint32_t bit = (R / 2) >> r, h = bit >> 1;
    // slots of the quartet offsets h, bit, bit + h (disjoint from j's bits)
    const uint32_t oh = lds_phys(h), ob = lds_phys(bit), obh = lds_phys(bit + h);
    for (uint32_t f = threadIdx.x; f < E / 4; f += blockDim.x) {
      const uint32_t gi = f / RQ, q = f % RQ;
      const uint32_t qm = q & (h - 1);
      const uint32_t j = (gi << DEG) + ((q / h) * (2 * bit)) + qm;
      const uint32_t pj = lds_phys(j);
      const F e0 = U.get(pj), e1 = U.get(pj ^ oh), e2 = U.get(pj ^ ob), e3 = U.get(pj ^ obh);
      const F s0 = rr_add_nc(e0, e2), s1 = rr_add_nc(e1, e3);
      F a0, a1, b0, b1;
      if (h > 1) {
        F d0, d1, a1p, b1p;
        rr_mul2(rr_sub_nc<8>(e0, e2), PQ.get((size_t)(qm << r) << pq_shift), rr_sub_nc<8>(e1, e3),
                PQ.get((size_t)((qm + h) << r) << pq_shift), d0, d1);
        a0 = rr_reduce_q(rr_add_nc(s0, s1));
        b0 = rr_carry_seq(rr_add_nc(d0, d1));
        const F w2 = PQ.get((size_t)(qm << (r + 1)) << pq_shift);
        rr_mul2(rr_sub_nc<16>(s0, s1), w2, rr_sub_nc<4>(d0, d1), w2, a1p, b1p);
        a1 = a1p;
        b1 = b1p;
      } else {  // h = 1 (the pass's last step): qm = 0, only d1's twiddle w^(1 << r) is non-trivial
        const F d0 = rr_reduce_q(rr_sub_nc<8>(e0, e2));
        const F d1 = rr_mul(rr_sub_nc<8>(e1, e3), PQ.get((size_t)(1u << r) << pq_shift));
        // Left unreduced ("P-form", see the header): every consumer -- the
        // next pass's twiddle product or rr_store_std's reduce_q -- takes
        // limbs < 2^31.4 and values < 64 r.
        a0 = rr_add_nc(s0, s1);      // <= 10 r, limbs < 2^31
        a1 = rr_sub_nc<16>(s0, s1);  // <= 21 r, limbs < 2^30 + 2^30.6
        b0 = rr_add_nc(d0, d1);      // <= 2.3 r
        b1 = rr_sub_nc<4>(d0, d1);   // <= 5.2 r, limbs < 2^29 + 2^30.6
      }
      U.put(pj, a0);
      U.put(pj ^ oh, a1);
      U.put(pj ^ ob, b0);
      U.put(pj ^ obh, b1);
    }
    __syncthreads();
  }
  if (r < DEG) {  // odd DEG: last radix-2 round (bit = 1, trivial twiddles), outputs in the P-form
    for (uint32_t f = threadIdx.x; f < E / 2; f += blockDim.x) {
      const uint32_t p0 = lds_phys(2 * f);  // phys(2f + 1) = phys(2f) ^ 1
      const F u0 = U.get(p0), u1 = U.get(p0 ^ 1);
      U.put(p0, rr_add_nc(u0, u1));           // <= 5 r
      U.put(p0 ^ 1, rr_sub_nc<8>(u0, u1));    // <= 10.5 r, limbs < 2^29 + 2^30.6
    }
    __syncthreads();
  }

  // ---- store: y[(g - k) 2^DEG + k + j 2^lgp] = v[j] (natural order)
  {
    const uint64_t p = 1ull << lgp;
    const uint32_t lpp = lgp < log_g ? lgp : log_g;
    const uint32_t pp = 1u << lpp;
#pragma unroll
    for (int q = 0; q < NTT_EPT; q++) {
      const uint32_t f = threadIdx.x + q * blockDim.x;
      if (f >= E) break;
      const uint32_t kk = f & (pp - 1);
      const uint32_t jj = (f >> lpp) & (R - 1);
      const uint32_t gh = f >> (lpp + DEG);
      const uint32_t gi = (gh << lpp) + kk;
      const uint64_t g = g0 + gi;
      const uint64_t k = g & (p - 1);
      const size_t dst = ((g - k) << DEG) + k + (uint64_t)jj * p;
      const F v = U.get(lds_phys((gi << DEG) + bitrev(jj, DEG)));
      if constexpr (OUT_RR)
        RrPlanes<Q>::over(y, n).put(dst, v);  // P-form: the next pass multiplies it by its twiddle first
      else
        rr_store_std<Q>(y, dst, v);
    }
  }
}

// boundary-form table entries w R -> w R' as planes of exact canonical limbs
template <class Q>
__global__ void ntt_tab_to_rr_kernel(const Fp<typename Q::Base>* __restrict__ in, uint64_t cnt, uint4* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt) return;
  RrPlanes<Q>::over(out, cnt).put(i, rr_canon_lt2p(rr_reduce_q(rr_from_std<Q>(load(&in[i])))));
}

// Full inter-pass twiddle table of one pass: out[i * p + k] = w^((k i) << s),
// i < 2^deg, k < p = 2^lgp, s = log n - lgp - deg.
template <class P>
__global__ void ntt_fulltw_kernel(const Fp<P>* __restrict__ tw_lo, const Fp<P>* __restrict__ tw_hi, uint32_t lgp,
                                  uint32_t deg, uint32_t log_n, Fp<P>* __restrict__ out) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >> (lgp + deg)) return;
  const uint64_t k = idx & ((1ull << lgp) - 1), i = idx >> lgp;
  const uint64_t e = (k * i) << (log_n - lgp - deg);
  store(&out[idx], e ? twiddle(tw_lo, tw_hi, e) : Fp<P>::one());
}

// out[j] = w^(j << shift), j < count  (w given by value, Montgomery)
template <class P>
__global__ void ntt_powers_kernel(Fp<P> w, uint32_t shift, uint64_t count, Fp<P>* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  Fp<P> base = w;
  for (uint32_t s = 0; s < shift; s++) base = fsqr(base);  // base = w^(2^shift)
  Fp<P> r = Fp<P>::one();
  uint64_t e = j;
  while (e) {
    if (e & 1) r = fmul(r, base);
    e >>= 1;
    if (e) base = fsqr(base);
  }
  store(&out[j], r);
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
struct PassArgs {
  const void* x;
  void* y;
  const void* pq;
  uint32_t pq_shift;
  const void* tw_lo;
  const void* tw_hi;
  const void* twf;  // full table of this pass, or null
  uint32_t log_n, lgp;
  uint32_t batch = 1;  // transforms back to back (reduced-radix passes only)
};

// A/B knob: log2 elements per workgroup (ECG_NTT_TILE, default 10)
static uint32_t ntt_tile_log() {
  static uint32_t v = [] {
    const char* e = getenv("ECG_NTT_TILE");
    return e ? (uint32_t)atoi(e) : 10u;
  }();
  return v;
}
template <class P, int DEG, bool V1>
static hipError_t launch_pass(const PassArgs& a, hipStream_t s) {
  using F = Fp<P>;
  const uint32_t tile_log = V1 ? 10 : (DEG > ntt_tile_log() ? DEG : ntt_tile_log());  // elements per workgroup
  uint32_t log_g = tile_log - DEG;
  const uint32_t log_groups = a.log_n - DEG;
  if (log_g > log_groups) log_g = log_groups;
  const uint32_t E = 1u << (DEG + log_g);
  const uint64_t blocks = 1ull << (log_groups - log_g);
  const size_t lds = (size_t)2 * E * sizeof(uint4);
  uint32_t threads;
  if (V1) {
    threads = 256;
  } else {
    threads = E / NTT_EPT;
    if (threads < 64) threads = 64;
    if (threads > 1024) threads = 1024;
  }
  auto kern = V1 ? ntt_pass_v1_kernel<P, DEG> : ntt_pass_kernel<P, DEG>;
  static bool attr_set = false;  // > 64 KiB dynamic LDS needs an explicit opt-in
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(threads), lds, s, (const F*)a.x, (F*)a.y, (const F*)a.pq,
                     a.pq_shift, (const F*)a.tw_lo, (const F*)a.tw_hi, (const F*)a.twf, a.log_n, a.lgp, log_g);
  return hipGetLastError();
}

static bool ntt_xcd_runs() {  // XCD-aware tile order (A/B: ECG_NTT_XCD=0 keeps blockIdx order)
  static bool v = [] {
    const char* e = getenv("ECG_NTT_XCD");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Tables of the reduced-radix passes (planes): pq (cnt entries) and the full
// per-pass twiddles (twf_cnt entries over all passes, this pass at twf_off).
struct RrTables {
  const void* pq;
  uint32_t pq_cnt;
  const void* twf;
  uint64_t twf_cnt, twf_off;
};

template <class Q, int DEG, bool IN_RR, bool OUT_RR>
static hipError_t launch_pass_rr(const PassArgs& a, const RrTables& t, hipStream_t s) {
  const uint32_t tile_log = DEG > ntt_tile_log() ? DEG : ntt_tile_log();
  uint32_t log_g = tile_log - DEG;
  const uint32_t log_groups = a.log_n - DEG;
  if (log_g > log_groups) log_g = log_groups;
  const uint32_t E = 1u << (DEG + log_g);
  const uint64_t blocks = 1ull << (log_groups - log_g);
  const size_t lds = (size_t)E * RR_PLANE_BYTES;
  uint32_t threads = E / NTT_EPT;
  if (threads < 64) threads = 64;
  if (threads > NTT_RR_THREADS) return hipErrorInvalidValue;  // tiles of <= 4096 elements only
  auto kern = ntt_pass_rr_kernel<Q, DEG, IN_RR, OUT_RR>;
  static bool attr_set = false;  // > 64 KiB dynamic LDS needs an explicit opt-in
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const uint64_t grid = blocks * a.batch;
  uint32_t log_tiles = 0;
  while ((1ull << log_tiles) < blocks) log_tiles++;
  hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(threads), lds, s, (const uint4*)a.x, (uint4*)a.y,
                     (const uint4*)t.pq, t.pq_cnt, a.pq_shift, (const uint4*)t.twf, t.twf_cnt, t.twf_off, a.log_n,
                     a.lgp, log_g, (uint32_t)(ntt_xcd_runs() && grid >= 8 && grid % 8 == 0), log_tiles);
  return hipGetLastError();
}

template <class Q, int DEG>
static hipError_t launch_pass_rr_io(bool in_rr, bool out_rr, const PassArgs& a, const RrTables& t, hipStream_t s) {
  if (in_rr) return out_rr ? launch_pass_rr<Q, DEG, true, true>(a, t, s) : launch_pass_rr<Q, DEG, true, false>(a, t, s);
  return out_rr ? launch_pass_rr<Q, DEG, false, true>(a, t, s) : launch_pass_rr<Q, DEG, false, false>(a, t, s);
}

template <class Q>
static hipError_t launch_pass_rr_deg(int deg, bool in_rr, bool out_rr, const PassArgs& a, const RrTables& t,
                                     hipStream_t s) {
  switch (deg) {
    case 1: return launch_pass_rr_io<Q, 1>(in_rr, out_rr, a, t, s);
    case 2: return launch_pass_rr_io<Q, 2>(in_rr, out_rr, a, t, s);
    case 3: return launch_pass_rr_io<Q, 3>(in_rr, out_rr, a, t, s);
    case 4: return launch_pass_rr_io<Q, 4>(in_rr, out_rr, a, t, s);
    case 5: return launch_pass_rr_io<Q, 5>(in_rr, out_rr, a, t, s);
    case 6: return launch_pass_rr_io<Q, 6>(in_rr, out_rr, a, t, s);
    case 7: return launch_pass_rr_io<Q, 7>(in_rr, out_rr, a, t, s);
    case 8: return launch_pass_rr_io<Q, 8>(in_rr, out_rr, a, t, s);
    case 9: return launch_pass_rr_io<Q, 9>(in_rr, out_rr, a, t, s);
    case 10: return launch_pass_rr_io<Q, 10>(in_rr, out_rr, a, t, s);
    case 11: return launch_pass_rr_io<Q, 11>(in_rr, out_rr, a, t, s);
    case 12: return launch_pass_rr_io<Q, 12>(in_rr, out_rr, a, t, s);
    default: return hipErrorInvalidValue;
  }
}

static bool ntt_rr_enabled() {  // reduced-radix butterflies (A/B: ECG_NTT_RR=0 keeps the 32-bit-limb passes)
  static bool v = [] {
    const char* e = getenv("ECG_NTT_RR");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <class P, bool V1>
static hipError_t launch_pass_deg(int deg, const PassArgs& a, hipStream_t s) {
  switch (deg) {
    case 1: return launch_pass<P, 1, V1>(a, s);
    case 2: return launch_pass<P, 2, V1>(a, s);
    case 3: return launch_pass<P, 3, V1>(a, s);
    case 4: return launch_pass<P, 4, V1>(a, s);
    case 5: return launch_pass<P, 5, V1>(a, s);
    case 6: return launch_pass<P, 6, V1>(a, s);
    case 7: return launch_pass<P, 7, V1>(a, s);
    case 8: return launch_pass<P, 8, V1>(a, s);
    case 9: return V1 ? hipErrorInvalidValue : launch_pass<P, 9, false>(a, s);
    case 10: return V1 ? hipErrorInvalidValue : launch_pass<P, 10, false>(a, s);
    case 11: return V1 ? hipErrorInvalidValue : launch_pass<P, 11, false>(a, s);
    case 12: return V1 ? hipErrorInvalidValue : launch_pass<P, 12, false>(a, s);
    default: return hipErrorInvalidValue;
  }
}

static int ntt_variant() {
  static int v = [] {
    const char* e = getenv("ECG_NTT_VARIANT");
    return (e && e[0] == '1') ? 1 : 2;
  }();
  return v;
}

static bool ntt_full_twiddles() {  // per-pass full twiddle tables (A/B: ECG_NTT_FULLTW=0)
  static bool v = [] {
    const char* e = getenv("ECG_NTT_FULLTW");
    return !(e && e[0] == '0');
  }();
  return v;
}

static uint32_t ntt_max_deg() {  // largest radix exponent per pass (v2), tunable for A/B
  static uint32_t d = [] {
    const char* e = getenv("ECG_NTT_MAXDEG");
    int v = e ? atoi(e) : 10;
    return (uint32_t)(v < 2 ? 2 : v > 12 ? 12 : v);
  }();
  return d;
}

// Pass degrees: v2 splits log n into ceil(log n / maxdeg) balanced passes;
// v1 uses radix-2^8 passes like the reference (fft.rs:101-102).
static int plan_passes(uint32_t log_n, int variant, uint32_t* degs) {
  if (variant == 1) {
    int np = 0;
    for (uint32_t lgp = 0; lgp < log_n;) {
      const uint32_t d = log_n - lgp < 8 ? log_n - lgp : 8;
      degs[np++] = d;
      lgp += d;
    }
    return np;
  }
  const uint32_t md = ntt_max_deg();
  const int np = (int)((log_n + md - 1) / md);
  for (int k = 0; k < np; k++) degs[k] = log_n / np + ((uint32_t)k < log_n % np ? 1 : 0);
  return np;
}

template <class P, class Q>
static int ntt_run_t(ecg_ctx* ctx, int field_id, void* d_data, const uint64_t* omega, uint32_t log_n,
                     hipStream_t s, ecg_abort_cb abort_cb, void* user, uint32_t batch = 1) {
  using F = Fp<P>;
  const int variant = ntt_variant();
  uint32_t degs[40];
  const int np = plan_passes(log_n, variant, degs);
  uint32_t max_deg = 0;
  for (int k = 0; k < np; k++) max_deg = degs[k] > max_deg ? degs[k] : max_deg;

  const uint64_t n = 1ull << log_n;
  const uint64_t lo_cnt = 1ull << NTT_LO_BITS;
  const uint64_t hi_cnt = n > lo_cnt ? (n >> NTT_LO_BITS) : 1;
  const uint64_t pq_cnt = max_deg > 1 ? 1ull << (max_deg - 1) : 1;

  // full per-pass tables (passes after the first): sum of 2^(lgp + deg) <= 2n entries
  const bool full = ntt_full_twiddles() && log_n <= 28 && np > 1;
  // reduced-radix passes need the full tables (their twiddles are one load each)
  const bool rr = ntt_rr_enabled() && variant == 2 && (np == 1 || full) && (1u << (max_deg > ntt_tile_log() ? max_deg : ntt_tile_log())) <= 4 * NTT_RR_THREADS;
  // bytes per element between passes: the plane layout for the reduced-radix
  // passes, the boundary layout otherwise
  const size_t elem = rr ? RR_PLANE_BYTES : sizeof(F);
  if (batch > 1 && !rr) {  // batched launches are a reduced-radix feature: one transform at a time
    for (uint32_t b = 0; b < batch; b++)
      ECG_TRY((ntt_run_t<P, Q>(ctx, field_id, (F*)d_data + b * n, omega, log_n, s, abort_cb, user, 1)));
    return ECG_OK;
  }

  void *scratch = nullptr, *scratch2 = nullptr, *tables;
  if (np > 1 || variant == 1) ECG_TRY(ws_get(ctx, "ntt_scratch", batch * n * elem, &scratch));
  // odd pass counts (> 1) rotate through a second scratch buffer so the last
  // pass writes d_data directly (no copy back; HBM is plentiful); the
  // reduced-radix inner passes always rotate two (planes do not fit d_data)
  if (np > 1 && ((np & 1) || (rr && np > 2))) ECG_TRY(ws_get(ctx, "ntt_scratch2", batch * n * elem, &scratch2));
  ECG_TRY(ws_get(ctx, "ntt_tables", (pq_cnt + lo_cnt + hi_cnt) * sizeof(F), &tables));
  F* pq = (F*)tables;
  F* tw_lo = pq + pq_cnt;
  F* tw_hi = tw_lo + lo_cnt;

  F* twf[40] = {nullptr};
  uint64_t twf_off[40] = {0}, twf_tot = 0;
  if (full) {
    uint32_t lg = 0;
    for (int k = 0; k < np; k++) {
      if (k > 0) {
        twf_off[k] = twf_tot;
        twf_tot += 1ull << (lg + degs[k]);
      }
      lg += degs[k];
    }
    void* t;
    ECG_TRY(ws_get(ctx, "ntt_twf", twf_tot * sizeof(F), &t));
    for (int k = 1; k < np; k++) twf[k] = (F*)t + twf_off[k];
  }
  // the reduced-radix passes' twiddles: w R' as planes of exact canonical limbs
  void *pq_rr = nullptr, *twf_rr = nullptr;
  if (rr) {
    ECG_TRY(ws_get(ctx, "ntt_pq_rr", pq_cnt * RR_PLANE_BYTES, &pq_rr));
    if (full) ECG_TRY(ws_get(ctx, "ntt_twf_rr", twf_tot * RR_PLANE_BYTES, &twf_rr));
  }

  const bool cached = ctx->tw_fid == field_id && ctx->tw_log_n == log_n && ctx->tw_variant == variant &&
                      ctx->tw_full == (int)full + 2 * (int)rr &&
                      memcmp(ctx->tw_omega, omega, sizeof(ctx->tw_omega)) == 0;
  if (!cached) {
    F w;
    memcpy(w.v, omega, sizeof(w.v));
    // pq[j] = w^(j * (n >> max_deg)) (fft.rs:68-78); tw_lo[j] = w^j; tw_hi[j] = w^(j << 12)
    hipLaunchKernelGGL(ntt_powers_kernel<P>, dim3((uint32_t)((pq_cnt + 255) / 256)), dim3(256), 0, s, w,
                       log_n - max_deg, pq_cnt, pq);
    hipLaunchKernelGGL(ntt_powers_kernel<P>, dim3((uint32_t)((lo_cnt + 255) / 256)), dim3(256), 0, s, w, 0u,
                       lo_cnt, tw_lo);
    hipLaunchKernelGGL(ntt_powers_kernel<P>, dim3((uint32_t)((hi_cnt + 255) / 256)), dim3(256), 0, s, w,
                       (uint32_t)NTT_LO_BITS, hi_cnt, tw_hi);
    if (full) {
      uint32_t lg = 0;
      for (int k = 0; k < np; k++) {
        if (k > 0) {
          const uint64_t cnt = 1ull << (lg + degs[k]);
          hipLaunchKernelGGL(ntt_fulltw_kernel<P>, dim3((uint32_t)((cnt + 255) / 256)), dim3(256), 0, s, tw_lo,
                             tw_hi, lg, degs[k], log_n, twf[k]);
        }
        lg += degs[k];
      }
    }
    if (rr) {
      hipLaunchKernelGGL(ntt_tab_to_rr_kernel<Q>, dim3((uint32_t)((pq_cnt + 255) / 256)), dim3(256), 0, s, pq,
                         pq_cnt, (uint4*)pq_rr);
      if (full)
        hipLaunchKernelGGL(ntt_tab_to_rr_kernel<Q>, dim3((uint32_t)((twf_tot + 255) / 256)), dim3(256), 0, s,
                           twf[1], twf_tot, (uint4*)twf_rr);
    }
    ECG_HIP(hipGetLastError());
    ctx->tw_fid = field_id;
    ctx->tw_log_n = log_n;
    ctx->tw_variant = variant;
    ctx->tw_full = (int)full + 2 * (int)rr;
    memcpy(ctx->tw_omega, omega, sizeof(ctx->tw_omega));
  }

  kt_reset(ctx, "ntt_pass");
  // Single-pass v2 transforms (log n <= 12) have one workgroup reading every
  // element before any write: safe in place.  Otherwise ping-pong, arranged so
  // the last pass lands in d_data whenever the pass count is even.
  void* bufs[41];
  bufs[0] = d_data;
  for (int k = 1; k <= np; k++) {
    if (variant == 1) bufs[k] = (k & 1) ? scratch : d_data;       // ping-pong + copy back (fft.rs:126)
    else if (np == 1) bufs[k] = d_data;                            // one workgroup: in place
    else if (k == np) bufs[k] = d_data;                            // last pass lands in place
    else if (rr) bufs[k] = (k & 1) ? scratch : scratch2;           // planes: two scratches
    else if (np & 1) bufs[k] = (k & 1) ? scratch : scratch2;       // odd: rotate two scratches
    else bufs[k] = (k & 1) ? scratch : d_data;                     // even: ping-pong
  }
  uint32_t lgp = 0;
  for (int k = 0; k < np; k++) {
    if (abort_cb && abort_cb(user)) return ECG_ABORTED;  // fft.rs:94-98
    const PassArgs a{bufs[k], bufs[k + 1], pq, max_deg - degs[k], tw_lo, tw_hi, twf[k], log_n, lgp, batch};
    ECG_TRY(kt_begin(ctx, "ntt_pass", s));
    hipError_t e;
    if (rr) {
      const RrTables t{pq_rr, (uint32_t)pq_cnt, twf_rr, twf_tot, twf_off[k]};
      e = launch_pass_rr_deg<Q>((int)degs[k], k > 0, k + 1 < np, a, t, s);
    }
    else
      e = variant == 1 ? launch_pass_deg<P, true>((int)degs[k], a, s) : launch_pass_deg<P, false>((int)degs[k], a, s);
    ECG_HIP(e);
    ECG_TRY(kt_end(ctx, "ntt_pass", s));
    lgp += degs[k];
  }
  if (bufs[np] != d_data)
    ECG_HIP(hipMemcpyAsync(d_data, bufs[np], batch * n * sizeof(F), hipMemcpyDeviceToDevice, s));
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
            ecg_abort_cb abort_cb, void* user, uint32_t batch) {
  ECG_TRY(ntt_validate(field_id, log_n));
  if (batch == 0) return ECG_OK;
  switch (field_id) {
    case ECG_FIELD_BLS12_381_FR:
      return ntt_run_t<params::bls12_381_fr, params::bls12_381_fr_rr>(ctx, field_id, d_data, omega, log_n, s,
                                                                       abort_cb, user, batch);
    default:
      return ntt_run_t<params::bn254_fr, params::bn254_fr_rr>(ctx, field_id, d_data, omega, log_n, s, abort_cb,
                                                               user, batch);
  }
}

}  // namespace ecg
