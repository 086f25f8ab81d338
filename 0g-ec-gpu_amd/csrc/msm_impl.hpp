// Pippenger multi-scalar multiplication on G1 and G2 (BLS12-381, BN254) for
// gfx950: kernels and per-curve drivers (instantiated once per curve by
// msm_inst.hip; msm.hip dispatches on curve_id).
//
// Replaces the reference's POINT_multiexp kernels (ag-build/cl/multiexp.cl:62-264,
// multiexp_backup.cl:11-71) and SingleMultiexpKernel::multiexp's host driver
// (ec-gpu-proxy/src/multiexp.rs:135-236).  Semantics follow multiexp_cpu
// (multiexp_cpu.rs:244-367): out = sum_i s_i * P_i, compared in affine.
//
// Re-design:
//  1. msm_digits      one thread per term: s mod r, signed c-bit windows
//                     (digit in [-2^(c-1), 2^(c-1)], as multiexp.cl:95-119 but
//                     applied to every window, carry-propagated), emits
//                     (key = window*B + |d|-1, val = term | sign<<31).
//  2. radix sort      (key, val) pairs, grouping each window's terms by bucket
//                     (rocPRIM onesweep; one 2-pass sort per window block of
//                     window-padded keys, see KeyMap).  Replaces the reference's
//                     per-thread global-memory bucket RMW (multiexp_backup.cl:45-58).
//  3. msm_accumulate  fixed-length segments of SEG sorted entries per thread
//                     (every lane runs exactly SEG XYZZ mixed adds, 8M+2S, of
//                     gathered affine bases, negated for negative digits, with
//                     a one-ahead gather prefetch): perfect lane balance
//                     whatever the bucket-size distribution.  Interior runs
//                     are whole buckets and are stored; the first and last
//                     run of each segment leave keyed partial records.
//                     The dominant kernel: VALU-bound on v_mad_u64_u32.
//                     G1 runs it in the reduced-radix form (curve_rr.hpp) on
//                     bases converted to 128-B records (msm_rr_bases).
//  4. msm_combine     the same fixed-segment scheme over the records, level
//                     by level (32 records per thread, x16 fewer per level):
//                     log-depth for any bucket skew.  Buckets without terms
//                     keep the memset identity.
//  5. msm_reduce      per window, 2^(c-1)/LS segments of LS buckets: running
//                     sums (summation by parts, multiexp.cl:121-131); then
//                     msm_reduce_offset adds the small-scalar multiple
//                     (s LS) x (segment total).
//  6. msm_sum         tree-fold of segment partials to one sum per window.
//  7. host fold       Horner over windows (c doublings each) and the final
//                     affine normalisation on the host -- the reference GPU
//                     path's own split (multiexp.rs:221-233): a serial chain of
//                     ~256 doublings is ~25x faster on one CPU core than on one
//                     GPU lane (host_field.hpp).
#pragma once
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "curve.hpp"
#include "host_pool.hpp"
#include "curve_rr2.hpp"
#include "dispatch.hpp"
#include "host_field.hpp"

namespace ecg {

constexpr int MSM_THREADS = 256;
constexpr uint32_t MSM_TREE_K = 2;           // inputs per thread of the tree-sum kernel
constexpr double MSM_MEMORY_PADDING = 0.2;    // share of HBM left free (multiexp.rs:24)
constexpr uint32_t MSM_COMBINE_SEG_MAX = 32;  // records per thread in msm_combine (upper bound)

// Tunables (env overrides for A/B measurement in one build).
static uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* e = getenv(name);
  return e ? (uint32_t)strtoul(e, nullptr, 10) : dflt;
}
// An A/B knob that must lie in [lo, hi]: anything else (unset, garbage, out
// of range) keeps the default.
static uint32_t env_u32_in(const char* name, uint32_t dflt, uint32_t lo, uint32_t hi) {
  const char* e = getenv(name);
  if (!e || !*e) return dflt;
  char* end = nullptr;
  const unsigned long v = strtoul(e, &end, 10);
  return (*end == 0 && v >= lo && v <= hi) ? (uint32_t)v : dflt;
}
static uint32_t msm_red_seg() {  // buckets per reduction segment (0: plan_reduction picks)
  static uint32_t v = env_u32_in("ECG_MSM_RED_SEG", 0, 1, 1u << 16);
  return v;
}
// Records per thread in msm_combine: each level is a serial chain of that many
// adds, so the level count (log_seg of the records) matters less than the
// depth: 8 measured 0.3 ms faster than 32 at 2^23 (profiles/r02d/ab_env.log).
static uint32_t msm_combine_seg() {  // A/B: ECG_MSM_COMB_SEG
  static uint32_t v = [] {
    uint32_t x = env_u32("ECG_MSM_COMB_SEG", 8);
    return x < 4 ? 4u : x > MSM_COMBINE_SEG_MAX ? MSM_COMBINE_SEG_MAX : x;
  }();
  return v;
}
static bool msm_short_runs() {  // A/B switch: ECG_MSM_SHORT=0 sends every record through the combine levels
  static const bool v = env_u32("ECG_MSM_SHORT", 1) != 0;
  return v;
}
static uint32_t msm_acc_seg() {  // sorted entries per accumulation thread
  static uint32_t v = env_u32_in("ECG_MSM_ACC_SEG", 128, 16, 4096);
  return v;
}

static bool msm_pw_enabled() {  // A/B switch: ECG_MSM_PW=0 keeps one global sort
  static const bool v = env_u32("ECG_MSM_PW", 1) != 0;
  return v;
}
static bool msm_fold_rr_enabled() {  // A/B switch: ECG_MSM_FOLD_RR=0 folds batched tasks in 32-bit limbs
  static const bool v = env_u32("ECG_MSM_FOLD_RR", 1) != 0;
  return v;
}
#define ECG_MSM_FOLD_RR_ON msm_fold_rr_enabled()
static bool msm_pw_one_enabled() {  // A/B switch: ECG_MSM_PW1=0 sorts every block on its own
  static const bool v = env_u32("ECG_MSM_PW1", 1) != 0;
  return v;
}
static int msm_sort_cfg() {  // onesweep config of the per-block sorts (A/B: ECG_MSM_SORTCFG)
  static const int v = (int)env_u32_in("ECG_MSM_SORTCFG", 2, 0, 3);
  return v;
}

// rocPRIM onesweep radix sort of the u64 entries (key << 32 | value) over
// key bits [b0, b1) -- a keys-only sort of one 8-B array, measured 7% faster
// than the same bytes as (u32 key, u32 value) pairs (tools/sort_bench.hip,
// profiles/r02b/sort_bench.log).
// cfg 0: rocPRIM's tuned gfx950 config (8-bit digits); 1, 2: 10-bit digits
// (1024-thread blocks, 8 / 12 items per thread): 20-bit block keys in 2 passes.
using SortCfg10a = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;
using SortCfg10b = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 12>, rocprim::kernel_config<1024, 12>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;
static hipError_t msm_sort(int cfg, void* tmp, size_t& bytes, const uint64_t* ei, uint64_t* eo, size_t n, int b0,
                           int b1, hipStream_t s) {
  switch (cfg) {
    case 1: return rocprim::radix_sort_keys<SortCfg10a>(tmp, bytes, ei, eo, n, 32 + b0, 32 + b1, s);
    case 2: return rocprim::radix_sort_keys<SortCfg10b>(tmp, bytes, ei, eo, n, 32 + b0, 32 + b1, s);
    default: return rocprim::radix_sort_keys(tmp, bytes, ei, eo, n, 32 + b0, 32 + b1, s);
  }
}
ECG_HD uint64_t msm_entry(uint32_t key, uint32_t val) { return ((uint64_t)key << 32) | val; }

// The headline blocks' sort (c = 20, one block of < 2^32 entries per window)
// without onesweep's histogram pass: the two 10-bit places' global digit
// offsets -- offs[0, 1024) for key bits [0, 10), offs[1024, 2048) for [10,
// 20), exclusive scans of the digit counts -- come from the digits kernel
// (msm_digits_hist_kernel, msm_hist_scan_kernel), which counts every entry
// as it writes it; this driver runs rocPRIM's two onesweep iterations (the
// decoupled look-back scatter passes of SortCfg10b) on them, as
// radix_sort_onesweep_impl does after its own histogram and scan kernels.
// A rocPRIM-internal entry point (rocprim::detail, the ROCm install's
// headers): msm_sort stays the fallback and the A/B (ECG_MSM_FUSED_HIST=0).
static hipError_t msm_sort_fused(void* tmp, size_t& bytes, const uint64_t* ei, uint64_t* eo, unsigned int n,
                                 unsigned int* offs, hipStream_t s) {
  namespace rd = rocprim::detail;
  using Cfg = typename SortCfg10b::onesweep_config;
  using WCfg = rd::wrapped_radix_sort_onesweep_config<Cfg, uint64_t, rocprim::empty_type>;
  bool use_atomic = false;
  ROCPRIM_RETURN_ON_ERROR(rd::check_if_using_atomic_block_id(s, use_atomic));
  rd::target_arch arch;
  ROCPRIM_RETURN_ON_ERROR(rd::host_target_arch(s, arch));
  const rd::radix_sort_onesweep_config_params params = rd::dispatch_target_arch<WCfg, false>(arch);
  if (params.radix_bits_per_place != 10) return hipErrorInvalidValue;  // offs holds two 10-bit places
  const unsigned int per_block = params.sort.block_size * params.sort.items_per_thread;
  const unsigned int nlook = 1024u * ((n + per_block - 1) / per_block);
  auto run = [&](auto atomic_id) -> hipError_t {
    using Bid = rd::block_id_wrapper<unsigned int, decltype(atomic_id)::value>;
    unsigned int* offs_tmp;
    rd::onesweep_lookback_state* look;
    uint64_t* keys_tmp;
    typename Bid::id_type* bid_store;
    ROCPRIM_RETURN_ON_ERROR(rd::temp_storage::partition(
        tmp, bytes,
        rd::temp_storage::make_linear_partition(rd::temp_storage::ptr_aligned_array(&offs_tmp, 1024u),
                                                rd::temp_storage::ptr_aligned_array(&look, nlook),
                                                rd::temp_storage::ptr_aligned_array(&keys_tmp, n),
                                                rd::temp_storage::make_partition(&bid_store,
                                                                                 Bid::get_temp_storage_layout()))));
    if (tmp == nullptr || n == 0) return hipSuccess;
    Bid bid = Bid::create(bid_store);
    rocprim::empty_type* nv = nullptr;
    ROCPRIM_RETURN_ON_ERROR((rd::radix_sort_onesweep_iteration<Cfg, false>(
        ei, keys_tmp, eo, nv, nv, nv, n, offs, offs_tmp, look, true, false, rocprim::identity_decomposer{}, 32u, 52u,
        bid, s, false)));
    return rd::radix_sort_onesweep_iteration<Cfg, false>(ei, keys_tmp, eo, nv, nv, nv, n, offs + 1024, offs_tmp,
                                                         look, false, true, rocprim::identity_decomposer{}, 42u,
                                                         52u, bid, s, false);
  };
  return use_atomic ? run(std::true_type{}) : run(std::false_type{});
}
// A/B switch, off by default: ECG_MSM_FUSED_HIST=1 counts the digits in the
// digits kernel.  Measured a wash at 2^24 and 2^26 (profiles/r05/fused_hist_ab.log):
// the 13 histogram launches go (1.9 ms) but the digits kernel's LDS atomics
// cost as much (1.54 -> 3.4 ms) -- rocPRIM's histogram pass is bound by the
// same LDS atomics, not by re-reading the entries.
static bool msm_fused_hist_enabled() {
  static const bool v = env_u32("ECG_MSM_FUSED_HIST", 0) != 0;
  return v;
}

struct MsmPlan {
  uint32_t c;     // window bits
  uint32_t W;     // windows
  uint32_t B;     // buckets per window = 2^(c-1)
  uint32_t S;     // reduction segments per window
  uint32_t LS;    // buckets per segment
  uint32_t seg;   // sorted entries per accumulation thread
  uint32_t G;     // bucket groups = tasks * W  (one group per (task, window)); tasks with a window table
  uint32_t tab;   // window-table mode: bases in the table (0 = off); every window shares its task's buckets
  // window pieces (msm_piece_t, the grid split of ecg_msm_dist_grid): the
  // digits run over wd windows (the carry chain of the whole scalar) and only
  // windows [w0, w0 + W) are emitted; wd = 0 means W (every window)
  uint32_t wd;
  uint32_t w0;
  ECG_HD uint32_t fold_windows() const { return tab ? 1u : W; }  // window sums per task
  ECG_HD uint32_t digit_windows() const { return wd ? wd : W; }
};

// Task geometry.  A single MSM is one task (n_lines = n_chunks = 1).  The
// batched form is ag-cuda-ec's multiple_multiexp (ag-cuda-ec/src/multiexp.rs:
// 21-81, kernel ag-build/cl/multiexp.cl:215-262): n_lines lines of line_len
// bases share one row of line_len scalars; each line is cut into n_chunks
// chunks of clen = line_len / n_chunks terms (a remainder is ignored, as in
// multiexp.cl:230), and task (line, chunk) computes
//   sum_{i < clen} s[chunk*clen + i] * P[line*line_len + chunk*clen + i].
// Window blocks of one rank's share of the grid split (msm_grid_t): block i
// holds window w0 + i over terms [lo[i], lo[i] + len[i]) of the n-term row,
// padded to mp[i] entries (a multiple of the accumulation segment) at
// offset off[i] of the entry list.
constexpr uint32_t MSM_GRID_MAXB = 16;
struct GridBlocks {
  uint32_t nb;
  uint64_t total;
  uint64_t off[MSM_GRID_MAXB];
  uint64_t len[MSM_GRID_MAXB];
  uint64_t lo[MSM_GRID_MAXB];
  uint64_t mp[MSM_GRID_MAXB];
};

struct MsmGeom {
  uint32_t n_lines;
  uint32_t n_chunks;
  size_t line_len;
  size_t clen;
  uint32_t scalar_mont;  // scalars arrive as Montgomery Fr elements (to_bigint on device)
  const GridBlocks* grid = nullptr;  // host-side: the grid split's window blocks (one task, one line)
  uint32_t tasks() const { return n_lines * n_chunks; }
};

// Buckets per reduction segment (LS; S = ceil(B / LS) segments per group,
// the last one possibly shorter).  A segment's running sums are a chain of
// 2 LS dependent full adds and the kernel is VALU-bound at 2 waves per SIMD,
// so what matters is that every SIMD gets the same share: with LS = 64 a
// 2^26 MSM has 13 x 8192 segments = 1.63 waves per SIMD, i.e. half the SIMDs
// run two 128-step chains while the others idle for the second.  Below
// MSM_RED_THREADS segments (2 waves on each of the 1024 SIMDs) the groups'
// buckets are therefore cut into exactly that many equal segments (any
// length: the offset kernel multiplies by the segment's first index).  The
// target is one round of `waves` waves per SIMD -- the reduction kernels'
// occupancy (RedWaves): 2 for reduced-radix G1 points, 1 for G2, whose second
// round of segments would only double the offset kernel's scalar products
// (G2 2^22: msm_reduce_offset 2.1 ms at 2 rounds).
// ECG_MSM_RED_SEG pins LS (A/B).
constexpr uint32_t MSM_RED_THREADS = 2 * 1024 * 64;
static void plan_reduction(MsmPlan& pl, uint32_t waves = 2) {
  const uint32_t target = MSM_RED_THREADS / 2 * waves;
  uint32_t ls = msm_red_seg();
  if (!ls) {
    ls = 64;
    if ((double)pl.G * pl.B / 64 < target) {
      const uint32_t per_group = std::max(1u, target / pl.G);
      ls = (pl.B + per_group - 1) / per_group;
      // a few hundred thousand buckets cut into chains shorter than 8 spend
      // more on the per-segment offsets (~1.5 log2 B point ops each) than on
      // the running sums: one wave per SIMD of 8-bucket chains is faster
      // (2^20: 4.47 -> 4.26 ms, 2^22: 12.9 -> 12.5 ms, profiles/r02h); smaller
      // MSMs stay latency-optimal with the shortest chains (2^18 with 8-bucket
      // chains: 2.53 -> 2.67 ms)
      if (ls < 8 && (double)pl.G * pl.B >= (double)(1u << 19)) ls = 8;
    }
  }
  pl.LS = pl.B < ls ? pl.B : ls;
  pl.S = (pl.B + pl.LS - 1) / pl.LS;
}

// Window size minimising  n*W + W*B*4 + W*c*12 (+ the per-block sort term
// below) per task (bucket accumulation vs reduction vs window-fold adds; a
// reduction step is ~2 full adds, ~1.4x a mixed add).  nbits = scalar MODULUS_BIT_SIZE.  forced_c != 0 pins c.
static MsmPlan make_plan(size_t n, uint32_t nbits, uint32_t forced_c = 0) {
  if (!forced_c) forced_c = env_u32_in("ECG_MSM_C", 0, 2, 22);  // A/B: pin the single-MSM window
  double best = 1e300;
  MsmPlan pl{};
  for (uint32_t c = 1; c <= 22; c++) {
    uint32_t W = (nbits + 1 + c - 1) / c;
    double B = (double)(1u << (c - 1));
    double cost = (double)n * W + W * B * 4.0 + W * c * 12.0;
    // Window-padded keys that do not fit one 20-bit sort with the window id
    // (msm_core_impl) are sorted block by block: each block's launch tails and
    // its latency-bound share of the reduction cost ~0.5M mixed adds over the
    // one-sort form (2^23: c = 16 measured 2% faster than c = 19 in
    // profiles/r02h/c_sweep23.log; 2^24 and up keep c = 20).
    uint32_t wbits = 0;
    while ((1u << wbits) < W) wbits++;
    if (n >= ((size_t)1 << 16) && c + wbits > 20) cost += W * 0.5e6;
    if (forced_c ? c == forced_c : (c >= 2 && cost < best)) {
      best = cost;
      pl.c = c;
      pl.W = W;
    }
  }
  pl.B = 1u << (pl.c - 1);
  pl.seg = msm_acc_seg();
  pl.G = pl.W;
  pl.tab = 0;
  plan_reduction(pl);
  return pl;
}

// Window table (ecg_msm_prepare_table): row k of the table holds 2^(k c) P_i
// (record i W + k: the W rows of a base are adjacent, so a task's gathers stay
// inside its own bases' records -- rows of their own, 2.7 GB apart on the AMT
// shape, made every gather a TLB miss: 2.7x slower accumulation),
// so the digit of window k of term i is a digit of base row k, and all W
// windows of a task feed ONE set of 2^(c-1) buckets.  The W-fold bucket
// reduction and the Horner fold disappear, which moves the best window from
// c = 20 (13 windows at 2^26) to c = 24 (11 windows): 15% fewer mixed adds.
// Cost model per term: W mixed adds; per bucket ~5 (2 full adds + the combine
// and reduction launches: the AMT shape measures c = 11 fastest, 75.4 vs
// 77.6 ms at c = 12).
static uint32_t table_window_auto(size_t n, uint32_t nbits) {
  double best = 1e300;
  uint32_t bc = 2;
  for (uint32_t c = 2; c <= 25; c++) {
    const uint32_t W = (nbits + 1 + c - 1) / c;
    const double cost = (double)n * W + 5.0 * (double)(1u << (c - 1));
    if (cost < best) {
      best = cost;
      bc = c;
    }
  }
  return bc;
}
static uint32_t table_rows(uint32_t nbits, uint32_t c) { return (nbits + 1 + c - 1) / c; }
static MsmPlan make_tab_plan(uint32_t tasks, uint32_t nbits, uint32_t c, size_t stride) {
  MsmPlan pl{};
  pl.c = c;
  pl.W = table_rows(nbits, c);
  pl.B = 1u << (c - 1);
  pl.seg = msm_acc_seg();
  pl.G = tasks;
  pl.tab = (uint32_t)stride;
  plan_reduction(pl);
  return pl;
}

// ---------------------------------------------------------------------------
// 1. signed-digit decomposition
// ---------------------------------------------------------------------------
// One thread per scalar j of the row; the digits are emitted once per line
// (entry (w, line, j) -> key = group(line, chunk(j), w) * B + |d| - 1).
// Scalar j reduced into s[0..7] (s[8] = 0 pads the window reads): optional
// Montgomery -> canonical, then mod r.
template <class C>
ECG_DEV void load_scalar(const uint4* __restrict__ scalars, size_t j, uint32_t mont, uint32_t* s) {
  using FrP = typename C::FrParams;
  const uint4 lo = scalars[2 * j], hi = scalars[2 * j + 1];
  s[0] = lo.x; s[1] = lo.y; s[2] = lo.z; s[3] = lo.w;
  s[4] = hi.x; s[5] = hi.y; s[6] = hi.z; s[7] = hi.w;
  s[8] = 0;
  if (mont) {  // PrimeFieldRepr::to_bigint (ag-types/src/impls.rs:13) on device
    Fp<FrP> m;
#pragma unroll
    for (int k = 0; k < 8; k++) m.v[k] = s[k];
    m = from_mont(m);
#pragma unroll
    for (int k = 0; k < 8; k++) s[k] = m.v[k];
  }
  // reduce mod r (any 256-bit input; at most 2^256/r subtractions)
  for (int it = 0; it < 8; it++) {
    uint32_t t[8];
    int64_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      c = (int64_t)s[k] - Fp<FrP>::p32(k) + (c >> 32);
      t[k] = (uint32_t)c;
    }
    if ((c >> 32) & 1) break;  // s < r
#pragma unroll
    for (int k = 0; k < 8; k++) s[k] = t[k];
  }
}

// Signed digit of window w (carry in/out), d in [-2^(c-1), 2^(c-1)].
ECG_DEV int32_t window_digit(const uint32_t* s, uint32_t w, const MsmPlan& pl, uint32_t& carry) {
  const uint32_t mask = (1u << pl.c) - 1;
  const uint32_t half = 1u << (pl.c - 1);
  const uint32_t bit = w * pl.c;
  const uint32_t limb = bit >> 5, sh = bit & 31;
  uint32_t v = 0;
  if (limb < 8) {
    const uint64_t two = (uint64_t)s[limb] | ((uint64_t)s[limb + 1] << 32);
    v = (uint32_t)(two >> sh) & mask;
  }
  int32_t d = (int32_t)(v + carry);
  carry = 0;
  if (w + 1 < pl.digit_windows() && (uint32_t)d >= half) {
    d -= (int32_t)(1u << pl.c);
    carry = 1;
  }
  return d;
}

// Key layout of the sorted (key, value) entries.
//  * global (kc = 0): key = group*B + |d|-1, zero digits get the sentinel G*B;
//    one sort over every entry (bits [0, log2(G*B+1))).
//  * window-padded (kc = c): each (window, line) block of m entries is padded
//    to mpad (a multiple of the accumulation segment) and keyed
//    group << c | local, local = |d|-1 or the block sentinel B (zero digits and
//    padding).  Every block is sorted on its own over bits [0, c) -- for c = 20
//    two 10-bit onesweep passes instead of three 8-bit passes over 23 bits --
//    measured 4 ms faster at 2^26.  Blocks align with segments, so a segment
//    never spans two blocks.
struct KeyMap {
  uint32_t kc;        // 0 = global keys, else c
  uint32_t B;         // buckets per group
  uint32_t sentinel;  // global mode: the sentinel key G*B
  ECG_DEV bool sent(uint32_t k) const { return kc ? (k & B) != 0 : k >= sentinel; }  // KEY_END too
  ECG_DEV uint32_t bucket(uint32_t k) const { return kc ? (k >> kc) * B + (k & (B - 1)) : k; }
};

// One thread per scalar j of the row.  Every line of a batched MSM shares
// the scalar row (ag-cuda-ec/src/multiexp.rs:21-81), so its digits -- and
// hence the sorted order -- are the same for every line: the entries are
// emitted and sorted ONCE, entry (w, j) at w * mpad + j with
// key = (chunk(j) * W + w, |d| - 1) and value = j | sign, and the
// accumulation walks the sorted list once per line (base and bucket offsets
// per line).
// The entries of scalar j (j < mpad); HIST: each entry's 20-bit local key also
// counts in the per-window digit histograms hist[(w 2 + place) 1024 + digit]
// (LDS, msm_digits_hist_kernel; window-padded keys with c = 20 only).
template <class C, bool HIST>
ECG_DEV void msm_digits_one(const uint4* __restrict__ scalars, const MsmGeom& g, const MsmPlan& pl, size_t mpad,
                            const KeyMap& km, uint64_t* __restrict__ ents, size_t j, uint32_t* hist) {
  const size_t m = (size_t)g.n_chunks * g.clen;
  auto count = [&](uint32_t w, uint32_t local) {  // 16-bit counters, two per LDS word
    if constexpr (HIST) {
      const uint32_t b0 = (w * 2) * 1024 + (local & 1023u), b1 = (w * 2 + 1) * 1024 + (local >> 10);
      atomicAdd(&hist[b0 >> 1], 1u << ((b0 & 1) * 16));
      atomicAdd(&hist[b1 >> 1], 1u << ((b1 & 1) * 16));
    }
  };
  if (j >= m) {  // block padding (window-padded mode only): block sentinels
    for (uint32_t w = 0; w < pl.W; w++) {
      const size_t o = (size_t)w * mpad + j;
      ents[o] = msm_entry((w << km.kc) | km.B, 0);
      count(w, km.B);
    }
    return;
  }
  uint32_t s[9];
  load_scalar<C>(scalars, j, g.scalar_mont, s);
  const uint32_t chunk = g.n_chunks == 1 ? 0u : (uint32_t)(j / g.clen);
  uint32_t carry = 0;
  const uint32_t wd = pl.digit_windows();
  for (uint32_t wa = 0; wa < wd; wa++) {
    const int32_t d = window_digit(s, wa, pl, carry);
    if (wa < pl.w0) continue;  // a window piece emits windows [w0, w0 + W) only
    const uint32_t w = wa - pl.w0;
    if (w >= pl.W) break;
    const uint32_t mag = d < 0 ? (uint32_t)(-d) : (uint32_t)d;
    const uint32_t sign = d < 0 ? 0x80000000u : 0u;
    const size_t o = (size_t)w * mpad + j;
    // window table: every window of the task shares its buckets and reads row w
    // of base j, record j * W + w (the rows of a base sit together)
    const uint32_t grp = pl.tab ? chunk : chunk * pl.W + w;
    const uint32_t bidx = pl.tab ? (uint32_t)j * pl.W + w : (uint32_t)j;
    if (d == 0) {
      ents[o] = msm_entry(km.kc ? (grp << km.kc) | km.B : km.sentinel, 0);
      count(w, km.B);
    } else {
      ents[o] = msm_entry(km.kc ? (grp << km.kc) | (mag - 1) : grp * pl.B + (mag - 1), bidx | sign);
      count(w, mag - 1);
    }
  }
}

// One thread per scalar j of the row.  Every line of a batched MSM shares
// the scalar row (ag-cuda-ec/src/multiexp.rs:21-81), so its digits -- and
// hence the sorted order -- are the same for every line: the entries are
// emitted and sorted ONCE, entry (w, j) at w * mpad + j with
// key = (chunk(j) * W + w, |d| - 1) and value = j | sign, and the
// accumulation walks the sorted list once per line (base and bucket offsets
// per line).
template <class C>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_digits_kernel(const uint4* __restrict__ scalars, MsmGeom g, MsmPlan pl, size_t mpad, KeyMap km,
                      uint64_t* __restrict__ ents) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= mpad) return;
  msm_digits_one<C, false>(scalars, g, pl, mpad, km, ents, j, nullptr);
}

// The grid split's entries (msm_grid_t): entry t of block i is term
// lo[i] + t - off[i] in window w0 + i (its digit carries the chain of the
// windows below it), or the block sentinel past len[i].
template <class C>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_digits_grid_kernel(const uint4* __restrict__ scalars, MsmGeom g, MsmPlan pl, KeyMap km, GridBlocks gb,
                           uint64_t* __restrict__ ents) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= gb.total) return;
  uint32_t i = 0;
  while (i + 1 < gb.nb && t >= gb.off[i + 1]) i++;
  const size_t j = t - gb.off[i];
  if (j >= gb.len[i]) {
    ents[t] = msm_entry((i << km.kc) | km.B, 0);
    return;
  }
  const size_t term = gb.lo[i] + j;
  uint32_t s[9];
  load_scalar<C>(scalars, term, g.scalar_mont, s);
  uint32_t carry = 0;
  int32_t d = 0;
  for (uint32_t wa = 0; wa <= pl.w0 + i; wa++) d = window_digit(s, wa, pl, carry);
  const uint32_t mag = d < 0 ? (uint32_t)(-d) : (uint32_t)d;
  const uint32_t sign = d < 0 ? 0x80000000u : 0u;
  ents[t] = d == 0 ? msm_entry((i << km.kc) | km.B, 0) : msm_entry((i << km.kc) | (mag - 1), (uint32_t)term | sign);
}

// The same entries for the c = 20 window blocks (msm_sort_fused), each
// counted in its window's two 10-bit digit histograms as it is written:
// MSM_HIST_SCALARS scalars per 1024-thread workgroup into LDS counters (W x
// 8 KB), then one global atomic per non-zero counter into ghist -- the
// histogram pass rocPRIM's onesweep would run over every block's 2^26 entries
// again (0.14 ms per window at 2^26).  Counters are 16-bit, two per LDS word
// (W x 4 KB: three workgroups per CU), so a workgroup counts at most 2^15
// scalars (a counter never exceeds 2^15, whatever the digits).
constexpr uint32_t MSM_HIST_THREADS = 1024;
constexpr uint32_t MSM_HIST_SCALARS = 1u << 15;
template <class C>
__global__ void __launch_bounds__(MSM_HIST_THREADS)
    msm_digits_hist_kernel(const uint4* __restrict__ scalars, MsmGeom g, MsmPlan pl, size_t mpad, KeyMap km,
                           uint64_t* __restrict__ ents, uint32_t* __restrict__ ghist) {
  extern __shared__ uint32_t lhist[];
  const uint32_t nb = pl.W * 1024;  // words of two counters
  for (uint32_t i = threadIdx.x; i < nb; i += MSM_HIST_THREADS) lhist[i] = 0;
  __syncthreads();
  const size_t j0 = (size_t)blockIdx.x * MSM_HIST_SCALARS;
  const size_t j1 = j0 + MSM_HIST_SCALARS < mpad ? j0 + MSM_HIST_SCALARS : mpad;
  for (size_t j = j0 + threadIdx.x; j < j1; j += MSM_HIST_THREADS)
    msm_digits_one<C, true>(scalars, g, pl, mpad, km, ents, j, lhist);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += MSM_HIST_THREADS) {
    const uint32_t h = lhist[i];
    if (h & 0xffffu) atomicAdd(&ghist[2 * i], h & 0xffffu);
    if (h >> 16) atomicAdd(&ghist[2 * i + 1], h >> 16);
  }
}

// Exclusive scan of each 1024-bin histogram (one workgroup per (window,
// place)): the global digit offsets of msm_sort_fused.
template <int THREADS = 1024>  // a template: this header is included by one translation unit per curve
__global__ void __launch_bounds__(THREADS) msm_hist_scan_kernel(uint32_t* __restrict__ ghist) {
  using Scan = hipcub::BlockScan<uint32_t, THREADS>;
  __shared__ typename Scan::TempStorage ts;
  uint32_t* h = ghist + (size_t)blockIdx.x * THREADS;
  uint32_t v = h[threadIdx.x];
  Scan(ts).ExclusiveSum(v, v);
  h[threadIdx.x] = v;
}

// ---------------------------------------------------------------------------
// 3. bucket accumulation over fixed-length segments (dominant kernel)
// ---------------------------------------------------------------------------
// Thread t owns sorted entries [t*SEG, (t+1)*SEG) and runs exactly SEG XYZZ
// mixed adds, whatever the bucket-size distribution.  Runs strictly inside
// the segment (another key on both sides) are whole buckets and are stored
// directly.  The first and the last run -- which may continue in the
// neighbouring segments -- are forwarded as keyed partial records
// (rec[2t], rec[2t+1]); a single-run segment forwards its sum plus an
// identity twin with the same key, so the record keys stay sorted with no
// holes.  msm_combine_kernel sums the records level by level.
constexpr uint32_t KEY_END = 0xffffffffu;

// Affine base [x, y] records as the accumulation gathers them: the boundary
// layout (2 Fq, packed) or, in the reduced-radix form, padded to whole 128-B
// lines (112 B -> 128 B for BLS12-381): an unaligned 112-B record straddles
// two lines for most bases, which doubled the gather traffic (PMC FETCH_SIZE).
template <class F>
struct BaseLayout {
  static constexpr size_t BYTES = 2 * sizeof(F);
};
template <class Q>
struct BaseLayout<FpR<Q>> {
  static constexpr size_t BYTES = (2 * sizeof(FpR<Q>) + 127) / 128 * 128;
};
template <class Q>
struct BaseLayout<FpR2<Q>> {  // G2: 4 NL words (224 B / 160 B) in two 128-B lines
  static constexpr size_t BYTES = (2 * sizeof(FpR2<Q>) + 127) / 128 * 128;
};
template <class F>
ECG_HD const F* base_ptr(const F* bases, size_t i) {
  return reinterpret_cast<const F*>(reinterpret_cast<const char*>(bases) + i * BaseLayout<F>::BYTES);
}
template <class F>
ECG_HD F* base_ptr(F* bases, size_t i) {
  return reinterpret_cast<F*>(reinterpret_cast<char*>(bases) + i * BaseLayout<F>::BYTES);
}

// r = c ? s : r limb by limb (Fp, FpR, Fp2).  A whole-struct `if (c) r = s`
// can become a copy through a selected pointer, i.e. via scratch memory.
template <class P>
ECG_DEV void limb_sel(Fp<P>& r, bool c, const Fp<P>& s) {
#pragma unroll
  for (int i = 0; i < Fp<P>::L; i++) r.v[i] = c ? s.v[i] : r.v[i];
}
template <class Q>
ECG_DEV void limb_sel(FpR<Q>& r, bool c, const FpR<Q>& s) {
  rr_sel(r, c, s);
}
template <class Q>
ECG_DEV void limb_sel(FpR2<Q>& r, bool c, const FpR2<Q>& s) {
  rr_sel(r, c, s);
}
template <class P>
ECG_DEV void limb_sel(Fp2<P>& r, bool c, const Fp2<P>& s) {
  limb_sel(r.c0, c, s.c0);
  limb_sel(r.c1, c, s.c1);
}

// Occupancy hint for the accumulate kernel (A/B: -DECG_ACC_WAVES=n sets
// amdgpu_waves_per_eu(n), i.e. a VGPR budget of 512/n per lane).
#ifdef ECG_ACC_WAVES
#define ECG_ACC_ATTR __attribute__((amdgpu_waves_per_eu(ECG_ACC_WAVES, ECG_ACC_WAVES)))
#else
#define ECG_ACC_ATTR
#endif

// Lines (batched MSM): thread ta works on segment t = ta / n_lines of line
// l = ta % n_lines -- the lanes of a wave walk the same sorted entries for
// neighbouring lines (same run boundaries, shared key loads) -- with base
// offset l * line_len and bucket offset l * line_buckets; its records go to
// slot l * nseg + t, so the record keys stay sorted line-major.
struct AccLines {
  uint32_t n_lines;
  size_t line_len;      // bases per line
  uint32_t line_buckets;  // buckets per line (n_chunks * W * B)
};

template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_ACC_ATTR
    msm_accumulate_kernel(const F* __restrict__ bases, const uint64_t* __restrict__ ents, size_t total, KeyMap km,
                          uint32_t seg, size_t nseg,
                          AccLines ln, XYZZ<F>* __restrict__ buckets, XYZZ<F>* __restrict__ recs,
                          uint32_t* __restrict__ rkeys) {
  const size_t ta = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ta >= nseg * ln.n_lines) return;
  size_t t = ta;
  uint32_t l = 0;
  if (ln.n_lines > 1) {
    t = ta / ln.n_lines;
    l = (uint32_t)(ta - t * ln.n_lines);
  }
  const size_t slot = (size_t)l * nseg + t;
  const F* lb = base_ptr(bases, (size_t)l * ln.line_len);
  const uint32_t boff = l * ln.line_buckets;
  const size_t e0 = t * seg;
  const size_t e1 = e0 + seg < total ? e0 + seg : total;
  const XYZZ<F> zero = xyzz_zero<F>();
  const uint64_t en0 = ents[e0];
  uint32_t b = (uint32_t)(en0 >> 32);
  if (km.sent(b)) {  // all-zero-digit tail: no records
    store_xyzz(&recs[2 * slot], zero);
    store_xyzz(&recs[2 * slot + 1], zero);
    rkeys[2 * slot] = KEY_END;
    rkeys[2 * slot + 1] = KEY_END;
    return;
  }
  uint32_t v = (uint32_t)en0;
  Affine<F> P = load_affine(base_ptr(lb, v & 0x7fffffffu));
  XYZZ<F> acc = zero;
  bool first_run = true;
  for (size_t e = e0; e < e1; e++) {
    // one-ahead prefetch of the next entry and its base
    const bool more = e + 1 < e1;
    const uint64_t enn = more ? ents[e + 1] : msm_entry(KEY_END, 0);
    const uint32_t kn = (uint32_t)(enn >> 32);
    const uint32_t vn = (uint32_t)enn;
    const bool last = km.sent(kn);  // end of segment or of the block's non-zero digits
    Affine<F> Pn;
    if (!last) Pn = load_affine(base_ptr(lb, vn & 0x7fffffffu));
    if (!aff_is_identity(P)) {  // GpuRepr identity (impls.rs:52-54) contributes nothing
      const F ny = pa_neg_y(P.y);  // k p - y: one subtraction (lazy range)
      // per-limb select: a whole-struct `if (neg) P.y = ny` lets the compiler
      // copy through a selected pointer, i.e. via scratch memory
      limb_sel(P.y, (v >> 31) != 0, ny);
      acc = pa_add_affine(acc, P);
    }
    if (kn != b) {
      const uint32_t bi = km.bucket(b) + boff;
      if (first_run) {
        store_xyzz(&recs[2 * slot], acc);
        rkeys[2 * slot] = bi;
        if (last) {
          store_xyzz(&recs[2 * slot + 1], zero);
          rkeys[2 * slot + 1] = bi;
          return;
        }
        first_run = false;
      } else if (last) {
        store_xyzz(&recs[2 * slot + 1], acc);
        rkeys[2 * slot + 1] = bi;
        return;
      } else {
        store_xyzz(&buckets[bi], acc);  // interior run: a whole bucket
      }
      acc = zero;
      b = kn;
    }
    P = Pn;
    v = vn;
  }
}

// ---------------------------------------------------------------------------
// 4a. short record runs in one launch.  Every key's records are one contiguous
//     run (2 per accumulation segment, in sorted order), and a bucket spans a
//     few segments at most unless the scalars are skewed: with uniform digits
//     the runs are 1-4 records long.  Thread t walks the runs that overlap its
//     MSM_SHORT_SEG records: a run of <= MSM_SHORT_RUN records is summed by the
//     thread whose window holds its first record (reading past its window if
//     the run does) and stored as the bucket -- len - 1 full adds, where a
//     combine level adds every record -- and its records' keys become KEY_END
//     in kout, so the level-by-level combine below carries them as
//     identities.  A longer run keeps its keys and raises *long_runs; with no
//     long run every level returns at its first instruction.  Each thread
//     writes kout for its own window only.  The 9-12 latency-bound levels (a
//     chain of 8 full adds each) were 0.49 ms of a 2^20 MSM.
// ---------------------------------------------------------------------------
//     Latency pays for it below MSM_SHORT_MAX_RECS records (2^20 MSM: 4.44 ->
//     4.05 ms; 2^23 at 2^21 records: no change); at 2^26 (13.6M records) the
//     work is throughput-bound and this kernel's lanes idle beside the run
//     owners (3.0 ms against 2.6 ms for all 12 levels,
//     profiles/r03f/combine_short_ab.txt), so large MSMs keep the levels.
constexpr uint32_t MSM_SHORT_RUN = 16;
constexpr uint32_t MSM_SHORT_SEG = 4;
constexpr size_t MSM_SHORT_MAX_RECS_DEFAULT_LOG = 21;
static size_t msm_short_max_recs() {  // A/B: ECG_MSM_SHORT_LOG
  static const size_t v = (size_t)1 << env_u32_in("ECG_MSM_SHORT_LOG", MSM_SHORT_MAX_RECS_DEFAULT_LOG, 4, 31);
  return v;
}
template <class F>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_combine_short_kernel(const XYZZ<F>* __restrict__ rin, const uint32_t* __restrict__ kin, size_t n,
                             uint32_t sentinel, XYZZ<F>* __restrict__ buckets, uint32_t* __restrict__ kout,
                             uint32_t* __restrict__ long_runs) {
  const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * MSM_SHORT_SEG;
  if (i0 >= n) return;
  const size_t i1 = i0 + MSM_SHORT_SEG < n ? i0 + MSM_SHORT_SEG : n;
  uint32_t k = kin[i0];
  size_t s = i0;  // start of the run holding record i0 (searched MSM_SHORT_RUN + 1 back at most)
  while (s > 0 && kin[s - 1] == k && i0 - s <= MSM_SHORT_RUN) s--;
  bool raised = false;
  for (size_t i = i0; i < i1;) {
    size_t e = i + 1;  // one past the run's last record (searched until the run is known long)
    while (e < n && kin[e] == k && e - s <= MSM_SHORT_RUN) e++;
    const bool lng = e - s > MSM_SHORT_RUN;
    const bool live = k < sentinel;  // KEY_END runs are identities
    const size_t je = e < i1 ? e : i1;
    for (size_t j = i; j < je; j++) kout[j] = live && !lng ? KEY_END : k;
    if (live && lng) raised = true;
    if (live && !lng && s >= i0) {  // this window holds the run's first record
      XYZZ<F> acc = load_xyzz(&rin[s]);
#pragma unroll 1
      for (size_t j = s + 1; j < e; j++) acc = pa_add(acc, load_xyzz(&rin[j]));
      store_xyzz(&buckets[k], acc);
    }
    if (lng) {  // skip to the run's end inside the window (its keys stay)
      while (e < i1 && kin[e] == k) kout[e++] = k;
    }
    i = e;
    s = e;
    if (i < i1) k = kin[i];
  }
  if (raised) *long_runs = 1u;
}

// ---------------------------------------------------------------------------
// 4. record combine: the same fixed-segment scheme over keyed partials
//    (full XYZZ adds).  Interior runs are whole buckets; first/last runs go
//    to the next level (2 per segment), so each level shrinks the record
//    count by seg/2 and the depth is logarithmic in the largest bucket --
//    a bucket holding a large share of all terms (skewed scalars) costs
//    O(log) levels, not a serial walk.  The last level (one segment) stores
//    every run.  Buckets never written stay at the memset identity (ZZ = 0).
// ---------------------------------------------------------------------------
template <class F>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_combine_kernel(const XYZZ<F>* __restrict__ rin, const uint32_t* __restrict__ kin, size_t n,
                       uint32_t sentinel, uint32_t seg, int final_level, XYZZ<F>* __restrict__ buckets,
                       XYZZ<F>* __restrict__ rout, uint32_t* __restrict__ kout,
                       const uint32_t* __restrict__ long_runs) {
  // Record keys are bucket indices or KEY_END (identity records of all-zero
  // segments, and the records msm_combine_short_kernel already summed).  Runs
  // of one key are contiguous; KEY_END runs may sit between blocks
  // (window-padded mode), so they are carried along, never stored.
  if (long_runs && *long_runs == 0) return;  // every run was short: nothing left
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t e0 = t * seg;
  if (e0 >= n) return;
  const size_t e1 = e0 + seg < n ? e0 + seg : n;
  const XYZZ<F> zero = xyzz_zero<F>();
  uint32_t b = kin[e0];
  XYZZ<F> acc = zero;
  bool first_run = true;
  for (size_t e = e0; e < e1; e++) {
    const bool end = e + 1 == e1;
    const uint32_t kn = end ? KEY_END : kin[e + 1];
    if (b < sentinel) acc = pa_add(acc, load_xyzz(&rin[e]));
    if (end || kn != b) {
      if (final_level) {
        if (b < sentinel) store_xyzz(&buckets[b], acc);
        if (end) return;
      } else if (first_run) {
        store_xyzz(&rout[2 * t], acc);
        kout[2 * t] = b;
        if (end) {
          store_xyzz(&rout[2 * t + 1], zero);
          kout[2 * t + 1] = b;
          return;
        }
        first_run = false;
      } else if (end) {
        store_xyzz(&rout[2 * t + 1], acc);
        kout[2 * t + 1] = b;
        return;
      } else if (b < sentinel) {
        store_xyzz(&buckets[b], acc);
      }
      acc = zero;
      b = kn;
    }
  }
}

// ---------------------------------------------------------------------------
// 5. per-segment summation by parts
// ---------------------------------------------------------------------------
// Two kernels: the running sums, then the segment offsets (sgm LS) run_s.
// One point of each chain is parked in LDS between its uses (word-major, one
// column per lane: conflict-free): with run, acc, the loaded bucket and the
// add's temporaries all in VGPRs these kernels needed > 256 registers and ran
// at 1 wave/SIMD.
// Reduced-radix (G1) points: 2 waves/SIMD at the price of a small spill.
// The Fq2 (G2) points keep the compiler's choice: forcing 2 waves would
// spill ~600 B per lane.
template <class F>
struct RedWaves {
  static constexpr int value = 1;
};
template <class Q>
struct RedWaves<FpR<Q>> {
  static constexpr int value = 2;
};
#define ECG_RED_ATTR __attribute__((amdgpu_waves_per_eu(RedWaves<F>::value)))

template <class F>
struct LdsPoint {  // XYZZ<F> words of lane t at w[i * MSM_THREADS + t]
  uint32_t* w;
  static constexpr int NW = (int)(sizeof(XYZZ<F>) / 4);
  ECG_DEV void put(const XYZZ<F>& p) const {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&p);
#pragma unroll
    for (int i = 0; i < NW; i++) w[i * MSM_THREADS + threadIdx.x] = s[i];
  }
  ECG_DEV XYZZ<F> get() const {
    XYZZ<F> p;
    uint32_t* d = reinterpret_cast<uint32_t*>(&p);
#pragma unroll
    for (int i = 0; i < NW; i++) d[i] = w[i * MSM_THREADS + threadIdx.x];
    return p;
  }
};

// Several bucket arrays (slots, `slot_stride` buckets apart) hold the buckets
// of the passes of one MSM (msm_host_t): bucket j is their sum, added into the
// running sum slot by slot -- one reduction for every pass.
template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_reduce_kernel(const XYZZ<F>* __restrict__ buckets, MsmPlan pl, XYZZ<F>* __restrict__ partial,
                      XYZZ<F>* __restrict__ runs, uint32_t slots, size_t slot_stride) {
  __shared__ uint32_t lds[LdsPoint<F>::NW * MSM_THREADS];
  const LdsPoint<F> acc_l{lds};
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= pl.G * pl.S) return;
  const uint32_t w = id / pl.S, sgm = id % pl.S;
  const XYZZ<F>* bk = buckets + (size_t)w * pl.B + (size_t)sgm * pl.LS;
  const uint32_t len = min(pl.LS, pl.B - sgm * pl.LS);  // the last segment may be shorter
  XYZZ<F> run = xyzz_zero<F>();
  acc_l.put(xyzz_zero<F>());
  for (int j = (int)len - 1; j >= 0; j--) {
#pragma unroll 1
    for (uint32_t q = 0; q < slots; q++) run = pa_add(run, load_xyzz(&bk[q * slot_stride + j]));
    acc_l.put(pa_add(acc_l.get(), run));
  }
  // acc = sum_j (j+1) S_j ; run = sum_j S_j
  store_xyzz(&partial[id], acc_l.get());
  store_xyzz(&runs[id], run);
}

// partial[id] += (sgm LS) run_sgm  (segment offset of the bucket weights)
template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_reduce_offset_kernel(const XYZZ<F>* __restrict__ runs, MsmPlan pl, XYZZ<F>* __restrict__ partial) {
  __shared__ uint32_t lds[LdsPoint<F>::NW * MSM_THREADS];
  const LdsPoint<F> base{lds};
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= pl.G * pl.S) return;
  const uint32_t sgm = id % pl.S;
  if (sgm == 0) return;
  const uint32_t k = sgm * pl.LS;  // double-and-add from the MSB; the base waits in LDS
  const XYZZ<F> p = load_xyzz(&runs[id]);
  base.put(p);
  XYZZ<F> acc = p;
  for (int b = 30 - __builtin_clz(k); b >= 0; b--) {
    acc = pa_dbl(acc);
    if ((k >> b) & 1) acc = pa_add(acc, base.get());
  }
  store_xyzz(&partial[id], pa_add(load_xyzz(&partial[id]), acc));
}

// ---------------------------------------------------------------------------
// 6. tree fold of `cnt` consecutive points per group: workgroup b of group g
//    sums inputs [b * TREE_K * 256, (b+1) * TREE_K * 256): each thread adds
//    TREE_K of them, then the workgroup halves its 256 points level by level in
//    LDS -> one point per workgroup, out[g * wgs + b].  Depth TREE_K + 8 adds
//    per launch (a fan-in-32 serial chain per thread was 32 per launch and
//    latency-bound: 3 launches, 1.0 ms at 2^26).
// ---------------------------------------------------------------------------
template <class F>
struct LdsPoints {  // XYZZ<F> words of point i at w[k * MSM_THREADS + i]
  uint32_t* w;
  static constexpr int NW = (int)(sizeof(XYZZ<F>) / 4);
  ECG_DEV void put(uint32_t i, const XYZZ<F>& p) const {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&p);
#pragma unroll
    for (int k = 0; k < NW; k++) w[k * MSM_THREADS + i] = s[k];
  }
  ECG_DEV XYZZ<F> get(uint32_t i) const {
    XYZZ<F> p;
    uint32_t* d = reinterpret_cast<uint32_t*>(&p);
#pragma unroll
    for (int k = 0; k < NW; k++) d[k] = w[k * MSM_THREADS + i];
    return p;
  }
};

template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_tree_sum_kernel(const XYZZ<F>* __restrict__ in, uint32_t cnt, uint32_t wgs, XYZZ<F>* __restrict__ out) {
  extern __shared__ uint32_t lds_pts[];
  const LdsPoints<F> pts{lds_pts};
  const uint32_t g = blockIdx.x / wgs, b = blockIdx.x % wgs, t = threadIdx.x;
  const XYZZ<F>* src = in + (size_t)g * cnt;
  const uint32_t j0 = (b * MSM_THREADS + t) * MSM_TREE_K;
  XYZZ<F> acc = xyzz_zero<F>();
#pragma unroll 1
  for (uint32_t k = 0; k < MSM_TREE_K; k++)
    if (j0 + k < cnt) acc = pa_add(acc, load_xyzz(&src[j0 + k]));
  pts.put(t, acc);
  __syncthreads();
  // only as many LDS levels as this workgroup has inputs for (a second launch
  // over a few workgroup sums ran all 8 levels: 2^20, 8 sums per window)
  const uint32_t left = cnt - b * MSM_THREADS * MSM_TREE_K;
  const uint32_t active = left >= MSM_THREADS * MSM_TREE_K ? MSM_THREADS : (left + MSM_TREE_K - 1) / MSM_TREE_K;
  uint32_t top = 1;
  while (top < active) top <<= 1;
#pragma unroll 1
  for (uint32_t stride = top / 2; stride > 0; stride >>= 1) {
    if (t < stride) pts.put(t, pa_add(pts.get(t), pts.get(t + stride)));
    __syncthreads();
  }
  if (t == 0) store_xyzz(&out[blockIdx.x], pts.get(0));
}

// 6b. Segment offsets by bits (one-task MSMs).  The offsets of step 5 are
//     sum_s (s LS) R_s = LS sum_k 2^k T_k,  T_k = sum_{s : bit k of s set} R_s,
//     k < KB = ceil(log2 S): KB plain tree sums, no point doubling on the
//     device; the host applies LS 2^k while it folds the windows
//     (msm_host_fold_bits).  Where msm_reduce_offset_kernel ran a double-and-
//     add of ~log2(B) dependent doublings per segment (latency-bound below
//     2^23: 0.58 ms of a 2^20 MSM; 28 point ops per segment at 2^26), the bit
//     sums cost KB S / 2 adds in trees of depth ~log2(S).  One launch also sums
//     A = sum_s A_s: group g = w (KB + 1) + k sums T_k of window w for k < KB,
//     and A for k = KB.  T_k's i-th input is segment
//     ((i >> k) << (k + 1)) | 2^k | (i mod 2^k), i < 2^(KB-1) (those >= S are
//     the identity).  Workgroup b of a group sums inputs [b 256 K, (b+1) 256 K),
//     K serially per thread, then log2(256) LDS levels.  Every add here waits
//     for the previous one (~15 us for a full add at this occupancy), so the
//     launch is sized by K (offset_bits_k) to ~one workgroup per CU.
//     Lane pairs (pp_add) do not pay here, capped at 2 waves/SIMD of
//     registers or not: 0.36 ms single against 0.38-0.41 ms paired at 2^20
//     (profiles/r04/tail_pairs_trace.txt, bits_pairs_trace.txt).
template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_offset_bits_kernel(const XYZZ<F>* __restrict__ partial, const XYZZ<F>* __restrict__ runs, uint32_t S,
                           uint32_t KB, uint32_t K, uint32_t wgs, XYZZ<F>* __restrict__ out) {
  extern __shared__ uint32_t lds_pts[];
  const LdsPoints<F> pts{lds_pts};
  const uint32_t g = blockIdx.x / wgs, b = blockIdx.x % wgs, t = threadIdx.x;
  const uint32_t w = g / (KB + 1), k = g % (KB + 1);
  const bool a_sum = k == KB;
  const XYZZ<F>* src = (a_sum ? partial : runs) + (size_t)w * S;
  const uint32_t cnt = a_sum ? S : (1u << (KB - 1));
  const uint32_t span = MSM_THREADS * K;
  if (b * span >= cnt) {  // this group has fewer inputs than the widest one: the identity
    if (t == 0) store_xyzz(&out[blockIdx.x], xyzz_zero<F>());
    return;
  }
  // input i = b span + q MSM_THREADS + t: a wave's lanes read neighbouring
  // segments at every step (coalesced), where a run of K per thread had each
  // lane stream its own region
  const uint32_t j0 = b * span + t;
  XYZZ<F> acc = xyzz_zero<F>();
#pragma unroll 1
  for (uint32_t q = 0; q < K; q++) {
    const uint32_t i = j0 + q * MSM_THREADS;
    if (i >= cnt) break;
    const uint32_t sg = a_sum ? i : (((i >> k) << (k + 1)) | (1u << k) | (i & ((1u << k) - 1)));
    if (sg < S) acc = pa_add(acc, load_xyzz(&src[sg]));
  }
  pts.put(t, acc);
  __syncthreads();
  const uint32_t left = cnt - b * span;
  const uint32_t active = left >= MSM_THREADS ? MSM_THREADS : left;  // threads holding an input
  uint32_t top = 1;
  while (top < active) top <<= 1;
#pragma unroll 1
  for (uint32_t stride = top / 2; stride > 0; stride >>= 1) {
    if (t < stride) pts.put(t, pa_add(pts.get(t), pts.get(t + stride)));
    __syncthreads();
  }
  if (t == 0) store_xyzz(&out[blockIdx.x], pts.get(0));
}

static uint32_t offset_bits(uint32_t S) {  // KB of msm_offset_bits_kernel
  uint32_t kb = 0;
  while ((1u << kb) < S) kb++;
  return kb;
}

// Inputs per thread of msm_offset_bits_kernel: enough that half a workgroup
// covers a bit group (2^(KB-1) inputs: K = 2^(KB-8)) and the A sum needs no
// second tree launch, within [2, 32].  The launch then has ~G (KB + 1)
// workgroups, under one per CU.  Measured at 2^20 (G = 16, S = 4096, KB = 12):
// K = 2 / 4 / 8 / 16 / 32 -> 0.67 / 0.54 / 0.45 / 0.38 / 0.59 ms for the
// offset and A sums (profiles/r04/offset_bits_k_ab.txt); the segment offsets
// and A tree of round 3 took 0.83 ms.  2^20 MSM 4.11 -> 4.05 ms with K = 16
// over K = 8; 2^26 (KB = 13) K = 32 within noise of 16
// (profiles/r04/tail_ls_k_ab.txt).  ECG_MSM_BITS_K pins K.
static uint32_t offset_bits_k(uint32_t S) {
  const uint32_t pinned = env_u32_in("ECG_MSM_BITS_K", 0, 1, 64);
  if (pinned) return pinned;
  const uint32_t kb = offset_bits(S);
  const uint32_t k = kb > 8 ? 1u << (kb - 8) : 2u;
  return std::min(32u, std::max(2u, k));
}

// 6b'. Offset-bit sums by a merge tree (one-task MSMs; the default in place
//     of msm_offset_bits_kernel).  Step 5 leaves per window and segment s < S
//     the partial P_s = sum_j (j + 1) S_{s LS + j} and the run R_s; the window
//     sum is A + LS sum_k 2^k T_k with A = sum_s P_s and T_k = sum_{s : bit k
//     of s set} R_s (step 6b; msm_host_fold_bits folds it).  Level j of the
//     tree holds, per block of 2^j consecutive segments, the block's SP = sum
//     P, SR = sum R and T_0 .. T_{j-1}; blocks L, R (R's segments above L's)
//     merge into
//        SP = SP_L + SP_R,  SR = SR_L + SR_R,  T_k = T_k^L + T_k^R (k < j),
//        T_j = SR_R:
//     j + 2 independent adds, one thread (or lane group) each, so every level
//     is ONE add deep: log2 S levels, ~3 S adds per window.  The bit-sum trees
//     of msm_offset_bits_kernel did KB S / 2 + S adds, K + 8 deep (24 at 2^20,
//     40 at 2^26).  Level j block t of window w: comps[(w nblk_j + t) (j + 2) +
//     i] = SP, SR, T_0, ...  The last level writes the host layout instead:
//     window w's T_0 .. T_{kb-1}, A at w (kb + 1) (the root's SR is not needed).
//     The upper levels have few adds, each a latency-bound chain under one wave
//     per SIMD: there a lane pair or quad shares each add (pp_add).
//     ECG_MSM_BITS_TREE=0 keeps msm_offset_bits_kernel (A/B).
static bool msm_bits_tree() {
  static const bool v = env_u32("ECG_MSM_BITS_TREE", 1) != 0;
  return v;
}
static uint32_t msm_bits_tree_lanes() {  // A/B: ECG_MSM_TREE_LANES = 1 (no sharing), 2 (up to pairs), 4 (up to quads)
  static const uint32_t v = env_u32_in("ECG_MSM_TREE_LANES", 4, 1, 4);
  return v;
}

// level 0 -> 1: segment pairs (2t, 2t + 1) of every window
template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_bits_leaf_kernel(const XYZZ<F>* __restrict__ partial, const XYZZ<F>* __restrict__ runs, uint32_t G,
                         uint32_t S, uint32_t fin, XYZZ<F>* __restrict__ out) {
  const uint32_t nb1 = (S + 1) / 2;
  const size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (size_t)G * nb1 * 2) return;
  const uint32_t comp = (uint32_t)(id & 1);  // 0: SP, 1: SR (and T_0)
  const size_t bt = id >> 1;
  const uint32_t w = (uint32_t)(bt / nb1), t = (uint32_t)(bt % nb1);
  const XYZZ<F>* src = (comp ? runs : partial) + (size_t)w * S + 2 * t;
  const XYZZ<F> l = load_xyzz(src);
  const bool has_r = 2 * t + 1 < S;
  const XYZZ<F> r = has_r ? load_xyzz(src + 1) : xyzz_zero<F>();
  if (fin) {  // S = 2: [T_0, A]
    if (comp == 0)
      store_xyzz(&out[(size_t)w * 2 + 1], has_r ? pa_add(l, r) : l);
    else
      store_xyzz(&out[(size_t)w * 2], r);
    return;
  }
  XYZZ<F>* o = out + bt * 3;
  store_xyzz(&o[comp], has_r ? pa_add(l, r) : l);
  if (comp == 1) store_xyzz(&o[2], r);  // T_0 = R_{2t+1}
}

// level j -> j + 1 (j >= 1): one add per (window, output block, component),
// on 2^LB lanes (PM: pp_add's lane sharing; LB = pp_lanes_log<PM>())
template <class F, int PM>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_bits_merge_kernel(const XYZZ<F>* __restrict__ in, uint32_t G, uint32_t nblk_in, uint32_t j, uint32_t fin,
                          XYZZ<F>* __restrict__ out) {
  constexpr uint32_t LB = pp_lanes_log<PM>();
  const uint32_t nblk_out = (nblk_in + 1) / 2, ci = j + 2;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t id = gid >> LB;  // the lanes of one add leave together
  if (id >= (size_t)G * nblk_out * ci) return;
  const bool lead = (gid & ((1u << LB) - 1)) == 0;
  const uint32_t comp = (uint32_t)(id % ci);
  const size_t bt = id / ci;  // (w, t) of the output block
  const uint32_t t = (uint32_t)(bt % nblk_out), w = (uint32_t)(bt / nblk_out);
  if (fin && comp == 1) {  // the root's SR is not needed, only T_j = SR_R
    if (lead) {
      const bool has_r = 2 * t + 1 < nblk_in;
      const XYZZ<F> r = has_r ? load_xyzz(&in[((size_t)w * nblk_in + 2 * t + 1) * ci + 1]) : xyzz_zero<F>();
      store_xyzz(&out[(size_t)w * (j + 2) + j], r);
    }
    return;
  }
  const XYZZ<F>* L = in + ((size_t)w * nblk_in + 2 * t) * ci;
  const bool has_r = 2 * t + 1 < nblk_in;  // uniform over the add's lanes
  const XYZZ<F> l = load_xyzz(&L[comp]);
  XYZZ<F> v = l, r = xyzz_zero<F>();
  if (has_r) {
    r = load_xyzz(&L[ci + comp]);
    v = pp_add<PM>(l, r);
  }
  // every lane of the group stores the same point: a lane-0-only store let
  // the compiler sink the lane exchanges of the result past the branch (the
  // G2 quad form returned a wrong point there, tests/test_gpu_g2.py)
  if (fin) {  // host layout [T_0 .. T_j, A]
    XYZZ<F>* o = out + (size_t)w * (j + 2);
    store_xyzz(&o[comp == 0 ? j + 1 : comp - 2], v);
  } else {
    XYZZ<F>* o = out + bt * (j + 3);
    store_xyzz(&o[comp], v);
    if (comp == 1) store_xyzz(&o[j + 2], r);  // T_j = SR_R
  }
}

// A few points per group (batched MSMs: 2 reduction segments per (task,
// window)): one thread per group adds them serially.  A tree-sum workgroup per
// group would run 8 LDS levels of adds for 2 inputs (13.9 ms on the AMT shape,
// 327680 workgroups).
constexpr uint32_t MSM_GROUP_SERIAL = 16;
template <class F>
__global__ void __launch_bounds__(MSM_THREADS) ECG_RED_ATTR
    msm_group_sum_kernel(const XYZZ<F>* __restrict__ in, uint32_t cnt, uint32_t groups, XYZZ<F>* __restrict__ out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const XYZZ<F>* src = in + (size_t)g * cnt;
  XYZZ<F> acc = load_xyzz(&src[0]);
#pragma unroll 1
  for (uint32_t k = 1; k < cnt; k++) acc = pa_add(acc, load_xyzz(&src[k]));
  store_xyzz(&out[g], acc);
}

// ---------------------------------------------------------------------------
// reduced-radix pipeline (curve_rr.hpp): bases into the R' form before step 3,
// window sums back to the 32-bit-limb form after step 6
// ---------------------------------------------------------------------------
// boundary field of a pipeline field, and the conversion into it
template <class AF>
struct StdOf;
template <class Q>
struct StdOf<FpR<Q>> {
  using type = Fp<typename Q::Base>;
  static ECG_DEV FpR<Q> conv(const type& a) { return rr_from_std<Q>(a); }
};
template <class Q>
struct StdOf<FpR2<Q>> {
  using type = Fp2<typename Q::Base>;
  static ECG_DEV FpR2<Q> conv(const type& a) { return rr2_from_std<Q>(a); }
};

template <class AF>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_rr_bases_kernel(const typename StdOf<AF>::type* __restrict__ in, size_t n, uint32_t stride,
                        AF* __restrict__ out) {
  using F = typename StdOf<AF>::type;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Affine<F> a = load_affine(in + 2 * i);
  Affine<AF> r;
  if (aff_is_identity(a)) {  // GpuRepr identity stays all-zero (impls.rs:52-54)
    r.x = AF::zero();
    r.y = AF::zero();
  } else {
    r.x = StdOf<AF>::conv(a.x);
    r.y = StdOf<AF>::conv(a.y);
  }
  AF* rec = base_ptr(out, i * stride);  // stride > 1: one row of an interleaved window table
  store_affine(rec, r);
  // zero the record's pad too: whole-line writes (a partial line costs a
  // read-modify-write; measured 3.3 -> 5.6 ms for this kernel without it)
  constexpr size_t body = (2 * sizeof(AF) + 15) / 16 * 16;  // store_affine writes whole 16-B vectors
  constexpr size_t pad = BaseLayout<AF>::BYTES - body;
  static_assert(pad % 16 == 0, "16-B vector stores");
  uint4* tail = reinterpret_cast<uint4*>(reinterpret_cast<char*>(rec) + body);
#pragma unroll
  for (size_t k = 0; k < pad / 16; k++) tail[k] = make_uint4(0, 0, 0, 0);
}

template <class F, class FS>
__global__ void msm_sums_to_std_kernel(const XYZZ<F>* __restrict__ in, uint32_t n, XYZZ<FS>* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_xyzz(&out[i], pa_to_std(load_xyzz(&in[i])));
}

// Batched form: the per-task Horner over its W window sums in the pipeline's
// reduced-radix point form, before the conversion.  The fold is a
// latency-bound chain of c (W - 1) doublings -- 1024 tasks are 16 waves on
// 1024 SIMDs, each wave alone on its SIMD -- so on G1 a lane quad (PM = 4)
// or pair (PM = 1) takes each task: pp_dbl / pp_add share every operation's
// products and a wave issues fewer instructions per doubling.
template <class F, int PM>
__global__ void __launch_bounds__(64)
    msm_fold_rr_kernel(const XYZZ<F>* __restrict__ sums, uint32_t nw, uint32_t c, uint32_t tasks,
                       XYZZ<F>* __restrict__ out) {
  constexpr uint32_t PB = pp_lanes_log<PM>();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t t = g >> PB;
  if (t >= tasks) return;  // the lanes of a task leave together
  XYZZ<F> acc = load_xyzz(&sums[(size_t)t * nw + nw - 1]);
  for (int w = (int)nw - 2; w >= 0; w--) {
    for (uint32_t k = 0; k < c; k++) acc = pp_dbl<PM>(acc);
    acc = pp_add<PM>(acc, load_xyzz(&sums[(size_t)t * nw + w]));
  }
  store_xyzz(&out[t], acc);  // every lane of the task holds acc (see msm_bits_merge_kernel)
}
static uint32_t msm_fold_lanes() {  // A/B: ECG_MSM_FOLD_PAIRS = 0 / 1 (one lane per task), 2 (pairs), 4 (quads)
  static const uint32_t v = env_u32_in("ECG_MSM_FOLD_PAIRS", 4, 0, 4);
  return v;
}

static bool msm_rr_enabled() {  // A/B switch: ECG_MSM_RR=0 runs the 32-bit-limb pipeline
  static const bool v = env_u32("ECG_MSM_RR", 1) != 0;
  return v;
}

// Coordinate field of the bucket pipeline: the reduced-radix Fq (G1) or Fq2
// (G2) form, else the boundary field (curves without an rr layout).
template <class C>
struct MsmField {
  using Q = typename RRof<typename C::FqParams>::Q;
  static constexpr bool rr = has_rr_form<C>() || has_rr2_form<C>();
  using type = std::conditional_t<has_rr_form<C>(), FpR<typename RR1of<typename C::FqParams>::Q>,
                                  std::conditional_t<has_rr2_form<C>(), FpR2<Q>, typename C::Fq>>;
};

// ---------------------------------------------------------------------------
// Synthetic bases P_i = (a + i*b) G  (bench/test input generator)
// ---------------------------------------------------------------------------
constexpr uint32_t GEN_BLOCK = 64;  // points per thread (batch-normalised)

template <class C>
ECG_DEV XYZZ<typename C::Fq> gen_mul(const uint32_t* k) {  // k (8 x u32 canonical) * G
  using F = typename C::Fq;
  Affine<F> g;
  from_u64_words(g.x, C::Gen::GX);
  from_u64_words(g.y, C::Gen::GY);
  XYZZ<F> acc = xyzz_zero<F>();
  for (int bit = 255; bit >= 0; bit--) {
    acc = xyzz_dbl(acc);
    if ((k[bit >> 5] >> (bit & 31)) & 1) acc = xyzz_add_affine(acc, g);
  }
  return acc;
}

template <class C>
__global__ void gen_step_kernel(Fp<typename C::FrParams> bc, typename C::Fq* __restrict__ q_aff) {
  using F = typename C::Fq;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Affine<F> a = xyzz_to_affine(gen_mul<C>(bc.v));
  store(&q_aff[0], a.x);
  store(&q_aff[1], a.y);
}

template <class C>
__global__ void __launch_bounds__(MSM_THREADS)
    gen_bases_kernel(Fp<typename C::FrParams> ac, Fp<typename C::FrParams> bc, size_t n,
                     const typename C::Fq* __restrict__ q_aff, typename C::Fq* __restrict__ out,
                     typename C::Fq* __restrict__ scratch) {
  using F = typename C::Fq;
  using S = Fp<typename C::FrParams>;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i0 = t * GEN_BLOCK;
  if (i0 >= n) return;
  const uint32_t cnt = (uint32_t)min((size_t)GEN_BLOCK, n - i0);
  // s0 = a + i0*b (mod r)
  const S am = to_mont(ac), bm = to_mont(bc);
  S im = S::zero();
  im.v[0] = (uint32_t)i0;
  im.v[1] = (uint32_t)(i0 >> 32);
  im = to_mont(im);
  S s0 = from_mont(fadd(am, fmul(bm, im)));
  XYZZ<F> P = gen_mul<C>(s0.v);
  Affine<F> Q = load_affine(q_aff);
  // walk and stash X, Y in out, ZZ, ZZZ and prefix products in scratch
  F pref = F::one();
  for (uint32_t k = 0; k < cnt; k++) {
    const size_t i = i0 + k;
    store(&out[2 * i], P.X);
    store(&out[2 * i + 1], P.Y);
    store(&scratch[3 * i], P.ZZ);
    store(&scratch[3 * i + 1], P.ZZZ);
    store(&scratch[3 * i + 2], pref);
    pref = fmul(pref, fmul(P.ZZ, P.ZZZ));
    P = xyzz_add_affine(P, Q);
  }
  F inv = finv(pref);
  for (int k = (int)cnt - 1; k >= 0; k--) {
    const size_t i = i0 + k;
    F zz = load(&scratch[3 * i]), zzz = load(&scratch[3 * i + 1]), pr = load(&scratch[3 * i + 2]);
    F d_inv = fmul(inv, pr);  // 1 / (ZZ*ZZZ) of point i
    inv = fmul(inv, fmul(zz, zzz));
    F x = fmul(load(&out[2 * i]), fmul(d_inv, zzz));
    F y = fmul(load(&out[2 * i + 1]), fmul(d_inv, zz));
    store(&out[2 * i], x);
    store(&out[2 * i + 1], y);
  }
}

// ---------------------------------------------------------------------------
// 7. batched form: per-task Horner fold over its W window sums + affine
//    normalisation, one thread per task (the single-MSM path folds on the
//    host instead, see msm_single_t).  Output: normalised Jacobian (x, y, 1)
//    or (0, 1, 0), the reference's G::Curve layout (multiexp.cl:259-261
//    writes one Jacobian per task).
// ---------------------------------------------------------------------------
template <class C>
__global__ void __launch_bounds__(64)
    msm_fold_kernel(const XYZZ<typename C::Fq>* __restrict__ sums, MsmPlan pl, uint32_t tasks,
                    typename C::Fq* __restrict__ out) {
  using F = typename C::Fq;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tasks) return;
  XYZZ<F> acc = xyzz_zero<F>();
  const int nw = (int)pl.fold_windows();
  for (int w = nw - 1; w >= 0; w--) {
    if (w != nw - 1)
      for (uint32_t k = 0; k < pl.c; k++) acc = xyzz_dbl<F, true>(acc);
    acc = xyzz_add<F, true>(acc, load_xyzz(&sums[(size_t)t * nw + w]));
  }
  acc = xyzz_canon(acc);
  const bool id = xyzz_is_zero(acc);
  Jac<F> j = jac_from_affine_norm(xyzz_to_affine(acc), id);
  store(&out[3 * (size_t)t], j.X);
  store(&out[3 * (size_t)t + 1], j.Y);
  store(&out[3 * (size_t)t + 2], j.Z);
}

// ---------------------------------------------------------------------------
// host drivers
// ---------------------------------------------------------------------------
static inline uint32_t blocks_for(size_t n, int threads) { return (uint32_t)((n + threads - 1) / threads); }

// How the (key, value) entries of one pass are sorted (ECG_SORT_* in ecgpu.h):
//  * GLOBAL:   global keys (group * B + bucket), one sort over every entry --
//              batched tasks, window tables, and passes below 2^16 terms;
//  * PW_ONE:   window-padded keys whose window id and bucket fit 20 bits
//              together (c + log2 W <= 20, i.e. c <= 16 up to 2^22 terms):
//              ONE 2-pass sort over all blocks;
//  * PW_BLOCK: window-padded keys, one 2-pass sort over the c-bit key per
//              window block (c = 20 from 2^24 terms: the headline plan).
// m = scalars of the row, line_groups = n_chunks * W.
static int msm_sort_mode(const MsmPlan& pl, size_t m, uint32_t n_chunks, uint32_t line_groups) {
  const bool pw = msm_pw_enabled() && !pl.tab && n_chunks == 1 && m >= ((size_t)1 << 16) &&
                  ((uint64_t)line_groups << pl.c) < 0xffffffffull;
  if (!pw) return ECG_SORT_GLOBAL;
  uint32_t wbits = 0;
  while ((1u << wbits) < line_groups) wbits++;
  return msm_pw_one_enabled() && pl.c + wbits <= 20 ? ECG_SORT_PW_ONE : ECG_SORT_PW_BLOCK;
}

// The plan a one-task MSM of n terms runs (ecg_msm_plan_info): the single
// MSM (window_bits = 0) or multiple_multiexp with one chunk and the window
// pinned to window_bits.
template <class C>
int msm_plan_info_t(size_t n, uint32_t window_bits, uint32_t* c, uint32_t* windows, int* sort_mode) {
  const MsmPlan pl = make_plan(n, (uint32_t)C::FrParams::BITS, window_bits);
  *c = pl.c;
  *windows = pl.W;
  *sort_mode = msm_sort_mode(pl, n, 1, pl.W);
  return ECG_OK;
}

// Steps 1-6 for one device pass: leaves pl.G window sums (lazy XYZZ) on the
// device and returns their address in *d_sums.
// AF = coordinate field of the bucket pipeline (C::Fq, or FpR<Q> for the
// reduced-radix form, whose bases are converted first).
// prepared: d_bases already holds the pipeline's base records
// (msm_prepare_t), so the per-call conversion is skipped.
// Phases of msm_core_impl: steps 1-4 (digits, sort, accumulation, combine)
// into bucket slot `slot`, and steps 5-6 (reduction over `slots` bucket
// slots, offsets, trees).  A pipelined MSM (msm_host_t) runs the first for
// each pass into its own slot and the second once.
// CORE_RESERVE only sizes the workspace (for the largest pass, before a
// pipeline starts: a buffer grown mid-pipeline would stall it).
enum MsmCorePhase { CORE_ALL = 0, CORE_ACC = 1, CORE_FIN = 2, CORE_RESERVE = 3 };
struct MsmSlots {
  uint32_t slot = 0;   // CORE_ACC: the bucket slot this pass fills (< slots)
  uint32_t slots = 1;  // the MSM's bucket slots (CORE_FIN reduces them all)
};

template <class C, class AF>
int msm_core_impl(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, const MsmGeom& g,
                  const MsmPlan& pl0, hipStream_t s, void** d_sums, bool prepared, bool* folded,
                  MsmCorePhase phase = CORE_ALL, MsmSlots sl = MsmSlots{}) {
  using F = AF;
  using X = XYZZ<F>;
  MsmPlan pl = pl0;  // reduction segments sized for this point form's occupancy
  plan_reduction(pl, RedWaves<F>::value);
  // one-task MSMs leave per window the A sum and the KB offset-bit sums
  // (the merge tree, or msm_offset_bits_kernel; folded on the host); batched
  // ones the window sums
  const bool bits = folded == nullptr;
  const bool tree = bits && msm_bits_tree() && pl.S >= 2;  // offset-bit sums by the merge tree (6b')
  const bool do_acc = phase == CORE_ALL || phase == CORE_ACC, do_fin = phase == CORE_ALL || phase == CORE_FIN;
  const size_t m = (size_t)g.n_chunks * g.clen;  // scalars consumed
  const uint32_t nb = pl.G * pl.B;
  const uint32_t sentinel = nb;
  // one line's entries (every line shares the scalar row; see msm_digits_kernel)
  const uint32_t line_groups = pl.G / g.n_lines;  // n_chunks * W
  // window-padded keys (KeyMap) when every (window, line) block is one group
  // and large enough for a sort of its own
  // the grid split's blocks always carry window-padded keys, sorted block by block
  const int sort_mode = g.grid ? ECG_SORT_PW_BLOCK : msm_sort_mode(pl, m, g.n_chunks, line_groups);
  const bool pw = sort_mode != ECG_SORT_GLOBAL;
  const GridBlocks* const gb = g.grid;  // grid split: blocks of their own lengths (window-padded keys)
  size_t mpad = pw ? (m + pl.seg - 1) / pl.seg * pl.seg : m;
  if (gb) {
    mpad = 0;
    for (uint32_t i = 0; i < gb->nb; i++) mpad = std::max<size_t>(mpad, gb->mp[i]);
  }
  const size_t total = gb ? gb->total : (size_t)pl.W * mpad;
  const KeyMap km{pw ? pl.c : 0u, pl.B, line_groups * pl.B};
  int key_bits = 1;
  while ((1ull << key_bits) <= km.sentinel) key_bits++;
  const size_t nseg = (total + pl.seg - 1) / pl.seg;        // segments of the sorted list
  const size_t nseg_all = nseg * g.n_lines;                 // accumulation threads (all lines)

  void *e0, *e1, *bk, *rc, *rk, *rc2, *rk2, *pa, *pb, *tmp;
  // the bucket slots, then one word: the long-run flag of msm_combine_short_kernel
  // every phase asks for all the MSM's slots: the grow-only workspace is
  // sized once, so slots filled by earlier passes are never reallocated
  const uint32_t nslots = sl.slots;
  ECG_TRY(ws_get(ctx, "msm_buckets", (size_t)nslots * nb * sizeof(X) + 256, &bk));
  X* const bk_all = (X*)bk;
  uint32_t* long_runs = (uint32_t*)((char*)bk + (size_t)nslots * nb * sizeof(X));
  if (phase == CORE_ACC) {
    // this pass's slot; the flag word sits after the last slot in use
    bk = (void*)(bk_all + (size_t)sl.slot * nb);
    long_runs = (uint32_t*)((char*)bk_all + (size_t)nslots * nb * sizeof(X));
  }
  ECG_TRY(ws_get(ctx, "msm_pa", (size_t)pl.G * pl.S * sizeof(X), &pa));
  // the merge tree's levels (6b'): odd ones in msm_tree1 (level 1, 3 points per
  // segment pair, is the largest), even ones in msm_tree2 (level 2: 4 points
  // per 4 segments); either may hold the last level's G (kb + 1) sums.  Every
  // phase sizes them.
  void *t1 = nullptr, *t2 = nullptr;
  if (tree) {
    const size_t fin_pts = (size_t)pl.G * (offset_bits(pl.S) + 1);
    ECG_TRY(ws_get(ctx, "msm_tree1", std::max((size_t)pl.G * ((pl.S + 1) / 2) * 3, fin_pts) * sizeof(X), &t1));
    ECG_TRY(ws_get(ctx, "msm_tree2", std::max((size_t)pl.G * ((pl.S + 3) / 4) * 4, fin_pts) * sizeof(X), &t2));
  }
  const uint32_t tree_span = MSM_TREE_K * MSM_THREADS;  // inputs per tree-sum workgroup
  ECG_TRY(ws_get(ctx, "msm_pb", ((size_t)pl.G * ((pl.S + tree_span - 1) / tree_span) + pl.G) * sizeof(X), &pb));
  // sort geometry (section 2 below)
  uint32_t wbits = 0;
  while ((1u << wbits) < line_groups) wbits++;
  const bool pw_one = sort_mode == ECG_SORT_PW_ONE;
  const int cfg = pw ? msm_sort_cfg() : 0;
  const size_t sort_n = pw && !pw_one ? mpad : total;  // one sort per block, or one sort of all blocks
  const int sort_bits = pw ? (int)(pw_one ? pl.c + wbits : pl.c) : key_bits;
  // the c = 20 window blocks (2^24 terms and up): digit histograms counted by
  // the digits kernel, onesweep without its histogram pass (msm_sort_fused)
  const bool fused = !gb && msm_fused_hist_enabled() && sort_mode == ECG_SORT_PW_BLOCK && pl.c == 20 && cfg == 2 &&
                     sort_n >= ((size_t)1 << 22) && sort_n < 0xffffffffull && pl.W * 8192u <= 160u * 1024u;
  void* hist = nullptr;
  if (do_acc || phase == CORE_RESERVE) {
  ECG_TRY(ws_get(ctx, "msm_e0", total * 8, &e0));
  ECG_TRY(ws_get(ctx, "msm_e1", total * 8, &e1));
  ECG_TRY(ws_get(ctx, "msm_recs", 2 * nseg_all * sizeof(X), &rc));
  ECG_TRY(ws_get(ctx, "msm_rkeys", 2 * nseg_all * 4, &rk));
  const uint32_t comb_seg = msm_combine_seg();
  const size_t nseg1 = (2 * nseg_all + comb_seg - 1) / comb_seg;
  ECG_TRY(ws_get(ctx, "msm_recs2", 2 * nseg1 * sizeof(X), &rc2));
  ECG_TRY(ws_get(ctx, "msm_rkeys2", 2 * nseg1 * 4, &rk2));
  size_t tmp_bytes = 0;
  if (fused) {
    ECG_HIP(msm_sort_fused(nullptr, tmp_bytes, (uint64_t*)e0, (uint64_t*)e1, (unsigned int)sort_n, nullptr, s));
    ECG_TRY(ws_get(ctx, "msm_hist", (size_t)pl.W * 2048 * 4, &hist));
  } else {
    ECG_HIP(msm_sort(cfg, nullptr, tmp_bytes, (uint64_t*)e0, (uint64_t*)e1, sort_n, 0, sort_bits, s));
  }
  ECG_TRY(ws_get(ctx, "msm_sort_tmp", tmp_bytes, &tmp));
  if (msm_short_runs()) {  // the short pass runs at the first level below msm_short_max_recs records
    void* ks;
    ECG_TRY(ws_get(ctx, "msm_rkeys_short", std::min(2 * nseg_all, msm_short_max_recs()) * 4, &ks));
  }
  if constexpr (!std::is_same<F, typename C::Fq>::value) {
    if (!prepared) {
      void* rb;
      ECG_TRY(ws_get(ctx, "msm_rr_bases", (size_t)g.n_lines * g.line_len * BaseLayout<F>::BYTES, &rb));
    }
  }
  if (phase == CORE_RESERVE) return ECG_OK;

  // buckets nobody writes (no term) stay the identity: all-zero XYZZ (ZZ = 0).
  // (Running this clear and the base conversion on a side stream, concurrent
  // with the digits and the sorts, measured no gain: all are HBM-bound.)
  ECG_HIP(hipMemsetAsync(bk, 0, (size_t)nb * sizeof(X), s));
  ECG_HIP(hipMemsetAsync(long_runs, 0, 4, s));
  const F* bases = (const F*)d_bases;
  if constexpr (!std::is_same<F, typename C::Fq>::value) {
    const size_t nb_in = (size_t)g.n_lines * g.line_len;  // every base a value can index
    if (!prepared) {
      void* rb;
      ECG_TRY(ws_get(ctx, "msm_rr_bases", nb_in * BaseLayout<F>::BYTES, &rb));
      hipLaunchKernelGGL(msm_rr_bases_kernel<F>, dim3(blocks_for(nb_in, MSM_THREADS)),
                         dim3(MSM_THREADS), 0, s, (const typename C::Fq*)d_bases, nb_in, 1u, (F*)rb);
      ECG_HIP(hipGetLastError());
      bases = (const F*)rb;
    }
  }

  if (fused) {
    const uint32_t lds = pl.W * 4096u;
    ECG_HIP(hipMemsetAsync(hist, 0, (size_t)pl.W * 2048 * 4, s));
    // > 64 KB of dynamic LDS needs the attribute (a host-side call; set per launch, whatever device)
    ECG_HIP(hipFuncSetAttribute((const void*)msm_digits_hist_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
    hipLaunchKernelGGL(msm_digits_hist_kernel<C>, dim3((uint32_t)((mpad + MSM_HIST_SCALARS - 1) / MSM_HIST_SCALARS)),
                       dim3(MSM_HIST_THREADS), lds, s, (const uint4*)d_scalars, g, pl, mpad, km, (uint64_t*)e0,
                       (uint32_t*)hist);
    ECG_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_hist_scan_kernel<1024>, dim3(pl.W * 2), dim3(1024), 0, s, (uint32_t*)hist);
    ECG_HIP(hipGetLastError());
  } else if (gb) {
    hipLaunchKernelGGL(msm_digits_grid_kernel<C>, dim3(blocks_for(total, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                       (const uint4*)d_scalars, g, pl, km, *gb, (uint64_t*)e0);
    ECG_HIP(hipGetLastError());
  } else {
    hipLaunchKernelGGL(msm_digits_kernel<C>, dim3(blocks_for(mpad, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                       (const uint4*)d_scalars, g, pl, mpad, km, (uint64_t*)e0);
    ECG_HIP(hipGetLastError());
  }

  // ---- group the (key, value) entries by bucket: rocPRIM onesweep radix sort
  // (an MSD counting sort with 10-bit coarse bins was measured 3x slower:
  // 13K bins leave ~0.15 entries per bin per tile, so its scatter cannot
  // coalesce -- onesweep's 8-bit digits exist for exactly that reason)
  // Window-padded keys whose window id and local key fit 20 bits together
  // (c <= 16 with 16 windows: up to 2^22 terms) are sorted in ONE 2-pass
  // sort over every block: the blocks already sit in window order and carry
  // the window in the key's high bits, so the stable sort leaves each block
  // where it was and yields exactly the per-block result.  Per-block sorts
  // of <= 2^22 entries took rocPRIM's small-input path (10 launches per block
  // at 2^20: 2.7 of the 7.1 ms MSM) or onesweep launch tails.
  if (gb) {  // one sort per block, each over its own padded length
    for (uint32_t i = 0; i < gb->nb; i++)
      ECG_HIP(msm_sort(cfg, tmp, tmp_bytes, (uint64_t*)e0 + gb->off[i], (uint64_t*)e1 + gb->off[i], gb->mp[i], 0,
                       sort_bits, s));
  }
  for (size_t o = 0, w = 0; !gb && o < total; o += sort_n, w++) {
    if (fused)
      ECG_HIP(msm_sort_fused(tmp, tmp_bytes, (uint64_t*)e0 + o, (uint64_t*)e1 + o, (unsigned int)sort_n,
                             (unsigned int*)hist + w * 2048, s));
    else
      ECG_HIP(msm_sort(cfg, tmp, tmp_bytes, (uint64_t*)e0 + o, (uint64_t*)e1 + o, sort_n, 0, sort_bits, s));
  }

  // one launch over every segment: per-block launches, each started as soon
  // as its block was sorted on a second stream, measured 6 ms slower at 2^26
  // (13 launch tails, and the concurrent sort slows the VALU-bound
  // accumulation by as much as it hides)
  ECG_TRY(kt_begin(ctx, "msm_accumulate", s));
  const AccLines ln{g.n_lines, pl.tab ? g.line_len * pl.W : g.line_len, line_groups * pl.B};
  hipLaunchKernelGGL(msm_accumulate_kernel<F>, dim3(blocks_for(nseg_all, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                     bases, (const uint64_t*)e1, total, km, pl.seg, nseg, ln, (X*)bk, (X*)rc,
                     (uint32_t*)rk);
  ECG_HIP(hipGetLastError());
  ECG_TRY(kt_end(ctx, "msm_accumulate", s));

  // combine the segment-edge partials level by level until fewer than
  // msm_short_max_recs records are left, then the short runs in one launch
  // and what is left level by level.  Large MSMs reach the short pass after
  // one or two throughput-bound levels: the record list then holds exactly
  // the buckets not yet stored (a level stores a bucket once all its records
  // met), so the short pass completes them as it does at the first level.
  // 2^26: levels 3-12 (0.68 ms, latency-bound from level 4 on) -> one short
  // pass (profiles/r04/combine_short_late_ab.txt).
  size_t nrec = 2 * nseg_all;
  X* rin = (X*)rc;
  uint32_t* kin = (uint32_t*)rk;
  X* rout = (X*)rc2;
  uint32_t* kout = (uint32_t*)rk2;
  const uint32_t* lflag = nullptr;
  for (;;) {
    if (!lflag && msm_short_runs() && nrec < msm_short_max_recs()) {
      void* ks;
      ECG_TRY(ws_get(ctx, "msm_rkeys_short", nrec * 4, &ks));
      hipLaunchKernelGGL(msm_combine_short_kernel<F>,
                         dim3(blocks_for((nrec + MSM_SHORT_SEG - 1) / MSM_SHORT_SEG, MSM_THREADS)), dim3(MSM_THREADS), 0,
                         s, (const X*)rin, (const uint32_t*)kin, nrec, sentinel, (X*)bk, (uint32_t*)ks, long_runs);
      ECG_HIP(hipGetLastError());
      kin = (uint32_t*)ks;
      lflag = long_runs;
    }
    const bool fin = nrec <= comb_seg;
    const size_t nthr = (nrec + comb_seg - 1) / comb_seg;
    hipLaunchKernelGGL(msm_combine_kernel<F>, dim3(blocks_for(nthr, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                       (const X*)rin, (const uint32_t*)kin, nrec, sentinel, comb_seg, fin ? 1 : 0, (X*)bk,
                       rout, kout, lflag);
    ECG_HIP(hipGetLastError());
    if (fin) break;
    nrec = 2 * nthr;
    std::swap(rin, rout);
    std::swap(kin, kout);
  }
  }  // do_acc
  if (!do_fin) return ECG_OK;

  uint32_t cnt = pl.S;
  uint32_t groups = pl.G;
  X* in = (X*)pa;
  X* out = (X*)pb;
  const size_t tree_lds = (size_t)LdsPoints<F>::NW * MSM_THREADS * 4;
  if (tree_lds > 64 * 1024) {  // G2 points (96 KiB per workgroup) need the opt-in
    ECG_HIP(hipFuncSetAttribute((const void*)msm_tree_sum_kernel<F>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)tree_lds));
    ECG_HIP(hipFuncSetAttribute((const void*)msm_offset_bits_kernel<F>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)tree_lds));
  }
  void* runs;
  ECG_TRY(ws_get(ctx, "msm_runs", (size_t)pl.G * pl.S * sizeof(X), &runs));
  hipLaunchKernelGGL(msm_reduce_kernel<F>, dim3(blocks_for((size_t)pl.G * pl.S, MSM_THREADS)),
                     dim3(MSM_THREADS), 0, s, (const X*)bk_all, pl, (X*)pa, (X*)runs, nslots, (size_t)nb);
  ECG_HIP(hipGetLastError());
  if (tree) {
    const uint32_t kb = offset_bits(pl.S);
    X* lv[2] = {(X*)t1, (X*)t2};
    uint32_t nblk = (pl.S + 1) / 2;
    hipLaunchKernelGGL(msm_bits_leaf_kernel<F>, dim3(blocks_for((size_t)pl.G * nblk * 2, MSM_THREADS)),
                       dim3(MSM_THREADS), 0, s, (const X*)pa, (const X*)runs, pl.G, pl.S, kb == 1 ? 1u : 0u,
                       lv[0]);
    ECG_HIP(hipGetLastError());
    int cur = 0;
    for (uint32_t j = 1; j < kb; j++) {
      const uint32_t nout = (nblk + 1) / 2;
      const size_t adds = (size_t)pl.G * nout * (j + 2);
      const uint32_t fin = j + 1 == kb ? 1u : 0u;
      // share each add over a lane quad / pair while that keeps the level
      // under one wave per SIMD (1024 SIMDs x 64 lanes)
      const uint32_t lanes = msm_bits_tree_lanes();
      bool done = false;
      if constexpr (QuadOps<F>::ok) {
        if (lanes >= 4 && adds * 4 <= 1024u * 64u) {
          hipLaunchKernelGGL((msm_bits_merge_kernel<F, 4>), dim3(blocks_for(adds * 4, MSM_THREADS)), dim3(MSM_THREADS),
                             0, s, (const X*)lv[cur], pl.G, nblk, j, fin, lv[cur ^ 1]);
          done = true;
        }
      }
      if constexpr (PairOps<F>::ok) {
        if (!done && lanes >= 2 && adds * 2 <= 1024u * 64u) {
          hipLaunchKernelGGL((msm_bits_merge_kernel<F, 1>), dim3(blocks_for(adds * 2, MSM_THREADS)), dim3(MSM_THREADS),
                             0, s, (const X*)lv[cur], pl.G, nblk, j, fin, lv[cur ^ 1]);
          done = true;
        }
      }
      if (!done)
        hipLaunchKernelGGL((msm_bits_merge_kernel<F, 0>), dim3(blocks_for(adds, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                           (const X*)lv[cur], pl.G, nblk, j, fin, lv[cur ^ 1]);
      ECG_HIP(hipGetLastError());
      cur ^= 1;
      nblk = nout;
    }
    in = lv[cur];  // per window T_0 .. T_{kb-1}, A
    groups = pl.G * (kb + 1);
    cnt = 1;
  } else if (bits) {
    const uint32_t kb = offset_bits(pl.S);
    const uint32_t K = offset_bits_k(pl.S);
    const uint32_t wgs = (pl.S + MSM_THREADS * K - 1) / (MSM_THREADS * K);
    groups = pl.G * (kb + 1);
    void* pbits;
    ECG_TRY(ws_get(ctx, "msm_pbits", (size_t)groups * wgs * sizeof(X), &pbits));
    hipLaunchKernelGGL(msm_offset_bits_kernel<F>, dim3(groups * wgs), dim3(MSM_THREADS), tree_lds, s, (const X*)pa,
                       (const X*)runs, pl.S, kb, K, wgs, (X*)pbits);
    ECG_HIP(hipGetLastError());
    in = (X*)pbits;
    cnt = wgs;
    void* pb2;
    ECG_TRY(ws_get(ctx, "msm_pbits2", ((size_t)groups * ((wgs + tree_span - 1) / tree_span) + groups) * sizeof(X),
                   &pb2));
    out = (X*)pb2;
  } else {
    hipLaunchKernelGGL(msm_reduce_offset_kernel<F>, dim3(blocks_for((size_t)pl.G * pl.S, MSM_THREADS)),
                       dim3(MSM_THREADS), 0, s, (const X*)runs, pl, (X*)pa);
    ECG_HIP(hipGetLastError());
  }
  if (!bits && cnt > 1 && cnt <= MSM_GROUP_SERIAL) {
    hipLaunchKernelGGL(msm_group_sum_kernel<F>, dim3(blocks_for(pl.G, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                       (const X*)in, cnt, pl.G, out);
    ECG_HIP(hipGetLastError());
    std::swap(in, out);
    cnt = 1;
  }
  while (cnt > 1) {
    const uint32_t wgs = (cnt + tree_span - 1) / tree_span;
    hipLaunchKernelGGL(msm_tree_sum_kernel<F>, dim3(groups * wgs), dim3(MSM_THREADS), tree_lds, s, (const X*)in,
                       cnt, wgs, out);
    ECG_HIP(hipGetLastError());
    X* t = in;
    in = out;
    out = t;
    cnt = wgs;
  }
  if constexpr (std::is_same<F, typename C::Fq>::value) {
    *d_sums = in;
  } else {  // window sums back to the 32-bit-limb form (canonical coordinates)
    uint32_t npts = pl.G;
    if (folded && pl.fold_windows() > 1 && ECG_MSM_FOLD_RR_ON) {  // batched: Horner per task first
      const uint32_t tasks = pl.G / pl.W;
      // lane quads / pairs while they leave each SIMD at most one wave
      bool paired = false;
      if constexpr (QuadOps<F>::ok) {
        if (msm_fold_lanes() >= 4 && tasks <= (1u << 14)) {
          hipLaunchKernelGGL((msm_fold_rr_kernel<F, 4>), dim3(blocks_for(4 * (size_t)tasks, 64)), dim3(64), 0, s,
                             (const X*)in, pl.W, pl.c, tasks, out);
          paired = true;
        }
      }
      if constexpr (PairOps<F>::ok) {
        if (!paired && msm_fold_lanes() >= 2 && tasks <= (1u << 15)) {
          hipLaunchKernelGGL((msm_fold_rr_kernel<F, 1>), dim3(blocks_for(2 * (size_t)tasks, 64)), dim3(64), 0, s,
                             (const X*)in, pl.W, pl.c, tasks, out);
          paired = true;
        }
      }
      if (!paired)
        hipLaunchKernelGGL((msm_fold_rr_kernel<F, 0>), dim3(blocks_for(tasks, 64)), dim3(64), 0, s, (const X*)in,
                           pl.W, pl.c, tasks, out);
      ECG_HIP(hipGetLastError());
      in = out;
      npts = tasks;
      *folded = true;
    }
    if (bits) npts = groups;
    void* st;
    if (bits) {
      // single MSMs: the window sums go straight into mapped pinned host memory
      // (the host folds them next).  A device buffer and a D2H copy left
      // ~0.2 ms between this kernel and the copy's blit at every size
      // (profiles/r04/msm_2p20_timeline.txt, profiles/r05/trace20).
      void* host;
      ECG_TRY(hws_get(ctx, "msm_sums_host", (size_t)npts * sizeof(XYZZ<typename C::Fq>), &host, &st));
    } else {
      ECG_TRY(ws_get(ctx, "msm_sums_std", (size_t)npts * sizeof(XYZZ<typename C::Fq>), &st));
    }
    hipLaunchKernelGGL((msm_sums_to_std_kernel<F, typename C::Fq>), dim3(blocks_for(npts, 64)), dim3(64), 0, s,
                       (const X*)in, npts, (XYZZ<typename C::Fq>*)st);
    ECG_HIP(hipGetLastError());
    *d_sums = st;
  }
  return ECG_OK;
}

// Steps 1-6; leaves pl.G window sums (lazy 32-bit-limb XYZZ) on the device.
// folded != nullptr (batched form): the reduced-radix pipeline may fold each
// task's windows itself (Horner, msm_fold_rr_kernel) and then leaves one sum
// per task and sets *folded.
template <class C>
int msm_core_t(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, const MsmGeom& g, const MsmPlan& pl,
               hipStream_t s, void** d_sums, bool prepared = false, bool* folded = nullptr,
               MsmCorePhase phase = CORE_ALL, MsmSlots sl = MsmSlots{}) {
  if (folded) *folded = false;
  if constexpr (MsmField<C>::rr) {
    if (msm_rr_enabled())
      return msm_core_impl<C, typename MsmField<C>::type>(ctx, d_bases, d_scalars, g, pl, s, d_sums, prepared,
                                                          folded, phase, sl);
  }
  return msm_core_impl<C, typename C::Fq>(ctx, d_bases, d_scalars, g, pl, s, d_sums, prepared, nullptr, phase, sl);
}

// Bytes per base in the pipeline's own layout: 128-B reduced-radix records
// (G1) or the [x, y] boundary layout (G2, or ECG_MSM_RR=0).
template <class C>
size_t msm_base_record_bytes() {
  if constexpr (MsmField<C>::rr) {
    if (msm_rr_enabled()) return BaseLayout<typename MsmField<C>::type>::BYTES;
  }
  return 2 * sizeof(typename C::Fq);
}
template <class C>
uint32_t msm_table_windows(uint32_t tab_c) {  // rows of a window table (G1 only)
  return C::EXT == 1 && tab_c >= 2 ? table_rows((uint32_t)C::FrParams::BITS, tab_c) : 0u;
}
template <class C>
uint32_t msm_table_auto(size_t n) {
  return C::EXT == 1 ? table_window_auto(n, (uint32_t)C::FrParams::BITS) : 0u;
}
template <class C>
size_t msm_prepared_bytes(size_t n, uint32_t tab_c) {
  return n * msm_base_record_bytes<C>() * (tab_c ? msm_table_windows<C>(tab_c) : 1u);
}

// Window-table rows (ecg_msm_prepare_table): row k+1 = 2^c row k.
// 1. c doublings per base (in the pipeline's point form AF), out as strict
//    32-bit-limb XYZZ;
// 2. batch normalisation to affine: one Fermat inversion per TAB_NORM_BLOCK
//    points (Montgomery's trick, as gen_bases_kernel);
// 3. the pipeline's record conversion (msm_rr_bases_kernel) into the row.
constexpr uint32_t TAB_NORM_BLOCK = 32;
template <class C, class AF>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_tab_dbl_kernel(const typename C::Fq* __restrict__ in, size_t n, uint32_t c,
                       XYZZ<typename C::Fq>* __restrict__ out) {
  using F = typename C::Fq;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Affine<F> a = load_affine(in + 2 * i);
  if (aff_is_identity(a)) {  // GpuRepr identity: every multiple is the identity
    store_xyzz(&out[i], xyzz_zero<F>());
    return;
  }
  if constexpr (std::is_same<AF, F>::value) {
    XYZZ<F> p = xyzz_dbl_affine(a);
    for (uint32_t k = 1; k < c; k++) p = xyzz_dbl(p);
    store_xyzz(&out[i], p);
  } else {
    XYZZ<AF> p = pa_from_std_rr<typename AF::Params>(xyzz_from_affine(a));
    for (uint32_t k = 0; k < c; k++) p = pa_dbl(p);
    store_xyzz(&out[i], xyzz_canon(pa_to_std(p)));
  }
}

template <class C>
__global__ void __launch_bounds__(MSM_THREADS)
    msm_tab_norm_kernel(const XYZZ<typename C::Fq>* __restrict__ pts, size_t n, typename C::Fq* __restrict__ pref,
                        typename C::Fq* __restrict__ out) {
  using F = typename C::Fq;
  const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * TAB_NORM_BLOCK;
  if (i0 >= n) return;
  const uint32_t cnt = (uint32_t)min((size_t)TAB_NORM_BLOCK, n - i0);
  F acc = F::one();
  for (uint32_t k = 0; k < cnt; k++) {
    const XYZZ<F> p = load_xyzz(&pts[i0 + k]);
    store(&pref[i0 + k], acc);
    if (!xyzz_is_zero(p)) acc = fmul(acc, fmul(p.ZZ, p.ZZZ));
  }
  F inv = finv(acc);
  for (int k = (int)cnt - 1; k >= 0; k--) {
    const size_t i = i0 + k;
    const XYZZ<F> p = load_xyzz(&pts[i]);
    Affine<F> r;
    if (xyzz_is_zero(p)) {
      r.x = F::zero();
      r.y = F::zero();
    } else {
      const F d_inv = fmul(inv, load(&pref[i]));  // 1 / (ZZ ZZZ) of point i
      inv = fmul(inv, fmul(p.ZZ, p.ZZZ));
      r.x = fmul(p.X, fmul(d_inv, p.ZZZ));
      r.y = fmul(p.Y, fmul(d_inv, p.ZZ));
    }
    store(&out[2 * i], r.x);
    store(&out[2 * i + 1], r.y);
  }
}

// upload_multiexp_bases (ag-cuda-ec/src/multiexp.rs:11-19): bases held on the
// device in the layout the bucket kernels gather, converted once instead of
// on every MSM over them (the conversion is ~2% of a 2^26 MSM).
// [x, y] -> records; record i goes to slot i * stride of d_out (stride = W:
// one row of an interleaved window table).
template <class C>
int msm_records_t(const void* d_bases, size_t n, void* d_out, hipStream_t s, uint32_t stride = 1) {
  if constexpr (MsmField<C>::rr) {
    if (msm_rr_enabled()) {
      using AF = typename MsmField<C>::type;
      hipLaunchKernelGGL(msm_rr_bases_kernel<AF>, dim3(blocks_for(n, MSM_THREADS)),
                         dim3(MSM_THREADS), 0, s, (const typename C::Fq*)d_bases, n, stride, (AF*)d_out);
      ECG_HIP(hipGetLastError());
      return ECG_OK;
    }
  }
  const size_t rb = 2 * sizeof(typename C::Fq);
  if (stride == 1)
    ECG_HIP(hipMemcpyAsync(d_out, d_bases, n * rb, hipMemcpyDeviceToDevice, s));
  else if (n)
    ECG_HIP(hipMemcpy2DAsync(d_out, stride * rb, d_bases, rb, rb, n, hipMemcpyDeviceToDevice, s));
  return ECG_OK;
}

template <class C, class AF>
int msm_table_rows_t(const void* d_bases, size_t n, uint32_t tab_c, void* d_out, hipStream_t s) {
  using F = typename C::Fq;
  const uint32_t W = msm_table_windows<C>(tab_c);
  const size_t rec = msm_base_record_bytes<C>();
  const size_t sl = std::min(n, (size_t)1 << 22);  // bases per slice (bounded scratch)
  void *pts = nullptr, *pref = nullptr, *aff[2] = {nullptr, nullptr};
  int rc = ECG_OK;
  auto fail = [&](hipError_t e) {
    (void)hipGetLastError();
    set_error("prepare_table: %s", hipGetErrorString(e));
    rc = e == hipErrorOutOfMemory ? ECG_ERR_NOMEM : ECG_ERR_HIP;
  };
  hipError_t e = hipMalloc(&pts, sl * sizeof(XYZZ<F>));
  if (e == hipSuccess) e = hipMalloc(&pref, sl * sizeof(F));
  if (e == hipSuccess) e = hipMalloc(&aff[0], sl * 2 * sizeof(F));
  if (e == hipSuccess) e = hipMalloc(&aff[1], sl * 2 * sizeof(F));
  if (e != hipSuccess) fail(e);
  for (size_t a = 0; rc == ECG_OK && a < n; a += sl) {
    const size_t len = std::min(sl, n - a);
    const F* cur = (const F*)d_bases + 2 * a;
    for (uint32_t k = 1; rc == ECG_OK && k < W; k++) {
      F* nxt = (F*)aff[k & 1];
      hipLaunchKernelGGL((msm_tab_dbl_kernel<C, AF>), dim3(blocks_for(len, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                         cur, len, tab_c, (XYZZ<F>*)pts);
      hipLaunchKernelGGL(msm_tab_norm_kernel<C>, dim3(blocks_for((len + TAB_NORM_BLOCK - 1) / TAB_NORM_BLOCK, 64)),
                         dim3(64), 0, s, (const XYZZ<F>*)pts, len, (F*)pref, nxt);
      if ((e = hipGetLastError()) != hipSuccess) {
        fail(e);
        break;
      }
      rc = msm_records_t<C>(nxt, len, (char*)d_out + ((size_t)a * W + k) * rec, s, W);
      cur = nxt;
    }
  }
  if (rc == ECG_OK && (e = hipStreamSynchronize(s)) != hipSuccess) fail(e);
  for (void* p : {pts, pref, aff[0], aff[1]})
    if (p) (void)hipFree(p);
  return rc;
}

template <class C>
int msm_prepare_t(ecg_ctx* ctx, const void* d_bases, size_t n, uint32_t tab_c, void* d_out, hipStream_t s) {
  (void)ctx;
  if (n == 0) return ECG_OK;
  // table row 0 = the bases themselves
  ECG_TRY(msm_records_t<C>(d_bases, n, d_out, s, tab_c ? msm_table_windows<C>(tab_c) : 1u));
  if (!tab_c) return ECG_OK;
  if constexpr (C::EXT == 1) {
    if constexpr (has_rr_form<C>()) {
      if (msm_rr_enabled())
        return msm_table_rows_t<C, FpR<typename RR1of<typename C::FqParams>::Q>>(d_bases, n, tab_c, d_out, s);
    }
    return msm_table_rows_t<C, typename C::Fq>(d_bases, n, tab_c, d_out, s);
  }
  set_error("prepare_table: window tables are built for the G1 curves only");
  return ECG_ERR_INVALID;
}

// The plan msm_core_impl runs for a one-task MSM (its reduction segments are
// sized for the pipeline point form's occupancy), and how many sums it leaves:
// per window the A sum and offset_bits(S) bit sums (msm_offset_bits_kernel).
template <class C>
MsmPlan msm_eff_plan(MsmPlan pl) {
  bool done = false;
  if constexpr (MsmField<C>::rr) {
    if (msm_rr_enabled()) {
      plan_reduction(pl, RedWaves<typename MsmField<C>::type>::value);
      done = true;
    }
  }
  if (!done) plan_reduction(pl, RedWaves<typename C::Fq>::value);
  return pl;
}
static inline uint32_t msm_single_sums(const MsmPlan& e) { return e.G * (offset_bits(e.S) + 1); }

template <class C>
host::HPoint<HostF<C>> msm_host_load(const XYZZ<typename C::Fq>& s) {
  host::HPoint<HostF<C>> p;
  static_assert(sizeof(p.X) == sizeof(s.X), "host/device coordinate layouts differ");
  memcpy(&p.X, &s.X, sizeof(p.X));
  memcpy(&p.Y, &s.Y, sizeof(p.Y));
  memcpy(&p.ZZ, &s.ZZ, sizeof(p.ZZ));
  memcpy(&p.ZZZ, &s.ZZZ, sizeof(p.ZZZ));
  p.X = host::hcanon(p.X);  // device values are in the lazy range [0, 2p]
  p.Y = host::hcanon(p.Y);
  p.ZZ = host::hcanon(p.ZZ);
  p.ZZZ = host::hcanon(p.ZZZ);
  return p;
}

// One-task fold of msm_offset_bits_kernel's sums (e = the effective plan):
// window w's sum is A_w + LS sum_k 2^k T_{w,k} (Horner over the bits, then LS
// by double-and-add), computed for all windows at once on the host pool's
// threads (each is ~30 independent point ops); then the Horner over windows
// (multiexp.rs:221-233) adds them into `total`.
template <class C>
void msm_host_fold_bits(const XYZZ<typename C::Fq>* sums, const MsmPlan& e, host::HPoint<HostF<C>>& total) {
  using HX = host::HPoint<HostF<C>>;
  const uint32_t kb = offset_bits(e.S), nw = e.fold_windows();
  std::vector<HX> win(nw);
  auto window = [&](uint32_t w) {
    const XYZZ<typename C::Fq>* g = sums + (size_t)w * (kb + 1);
    HX x = HX::zero();
    for (int k = (int)kb - 1; k >= 0; k--) x = host::hadd_pts(host::hdbl(x), msm_host_load<C>(g[k]));
    HX y = HX::zero();  // LS x
    for (int b = 31 - __builtin_clz(e.LS); b >= 0; b--) {
      y = host::hdbl(y);
      if ((e.LS >> b) & 1) y = host::hadd_pts(y, x);
    }
    win[w] = host::hadd_pts(msm_host_load<C>(g[kb]), y);
  };
  if (nw >= 4 && kb >= 4)
    HostPool::get().parallel_for(nw, [&](size_t w) { window((uint32_t)w); });
  else
    for (uint32_t w = 0; w < nw; w++) window(w);
  // Horner over the windows: c (W - 1) serial doublings, in Jacobian form
  // (2M + 5S each instead of XYZZ's 6M + 3S)
  using HJ = host::HJac<HostF<C>>;
  HJ acc = HJ::zero();
  for (int w = (int)nw - 1; w >= 0; w--) {
    for (uint32_t k = 0; k < e.c; k++) acc = host::hjac_dbl(acc);
    acc = host::hjac_add(acc, host::hjac_from_xyzz(win[w]));
  }
  // a window piece's first window is window w0 of the scalar: weight 2^(c w0)
  for (uint32_t k = 0; k < e.c * e.w0; k++) acc = host::hjac_dbl(acc);
  total = host::hadd_pts(total, host::hxyzz_from_jac(acc));
}

// The window sums of a single-task core call, on the host after s is drained.
// The reduced-radix pipeline wrote them into the mapped pinned buffer
// "msm_sums_host" already (msm_sums_to_std_kernel); the boundary-form pipeline
// (ECG_MSM_RR=0) leaves them in device memory at d_sums, so they are copied.
template <class X>
int msm_sums_to_host(ecg_ctx* ctx, const void* d_sums, size_t count, hipStream_t s, X** win) {
  const size_t bytes = count * sizeof(X);
  bool mapped = false;
  auto it = ctx->hws.find("msm_sums_host");
  if (it != ctx->hws.end() && it->second.ptr && it->second.bytes >= bytes) {
    void* dev = nullptr;
    ECG_HIP(hipHostGetDevicePointer(&dev, it->second.ptr, 0));
    mapped = dev == d_sums;
  }
  ECG_TRY(hws_get(ctx, "msm_sums_host", bytes, (void**)win));  // no growth when mapped
  if (!mapped) ECG_HIP(hipMemcpyAsync(*win, d_sums, bytes, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  return ECG_OK;
}

// One piece of the (window x term) grid of an n_plan-term MSM: windows
// [w0, w0 + nwin) of the n_plan-term plan over the m terms at d_bases /
// d_scalars (views at the piece's first term).  Returns the piece's partial,
// sum over its windows w and terms t of 2^(c w) d_w(s_t) P_t, normalised.
// Every rank of ecg_msm_dist_grid runs its pieces with the same plan (from
// n_plan), so the partials of all ranks add up to the whole MSM.
template <class C>
int msm_piece_t(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, size_t m, size_t n_plan, uint32_t w0,
                uint32_t nwin, uint64_t* out_jac, hipStream_t s, BaseForm bf) {
  using HX = host::HPoint<HostF<C>>;
  using X = XYZZ<typename C::Fq>;
  if (bf.tab_c) {
    set_error("multiexp: window pieces need plain prepared bases or [x, y] bases, not a window table");
    return ECG_ERR_INVALID;
  }
  MsmPlan pl = make_plan(n_plan, (uint32_t)C::FrParams::BITS);
  if (w0 + nwin > pl.W || nwin == 0 || m > 0x7fffffffull) {
    set_error("multiexp: window piece [%u, %u) outside the %u windows of the plan", w0, w0 + nwin, pl.W);
    return ECG_ERR_INVALID;
  }
  HX total = HX::zero();
  if (m > 0) {
    pl.wd = pl.W;
    pl.w0 = w0;
    pl.W = nwin;
    pl.G = nwin;
    plan_reduction(pl);  // the caller resets the msm_accumulate timer
    const MsmGeom g{1, 1, m, m, 0};
    void* d_sums;
    ECG_TRY(msm_core_t<C>(ctx, d_bases, d_scalars, g, pl, s, &d_sums, bf.prepared));
    const MsmPlan e = msm_eff_plan<C>(pl);
    X* win;
    ECG_TRY(msm_sums_to_host(ctx, d_sums, msm_single_sums(e), s, &win));
    msm_host_fold_bits<C>(win, e, total);
  }
  host::hto_jac_norm(total, out_jac);
  return ECG_OK;
}

// One rank's share of the grid split in ONE core call: windows [w0, w0 + nw)
// of the n-term plan -- window w0 over terms [lo_first, n) (or [lo_first,
// hi_last) when nw = 1), the middle windows over all n terms, window
// w0 + nw - 1 over [0, hi_last) -- as window blocks of their own lengths: one
// digits launch, one sort per block, one accumulation, one reduction and one
// host fold.  (msm_piece_t's core call per piece paid a partly filled
// accumulation round, a reduction and a scalar read per piece: DESIGN.md §7.)
template <class C>
int msm_grid_t(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, uint32_t w0, uint32_t nw,
               size_t lo_first, size_t hi_last, uint64_t* out_jac, hipStream_t s, BaseForm bf) {
  using HX = host::HPoint<HostF<C>>;
  using X = XYZZ<typename C::Fq>;
  if (bf.tab_c) {
    set_error("multiexp: the grid split needs plain prepared bases or [x, y] bases, not a window table");
    return ECG_ERR_INVALID;
  }
  MsmPlan pl = make_plan(n, (uint32_t)C::FrParams::BITS);
  if (nw == 0 || nw > MSM_GRID_MAXB || w0 + nw > pl.W || n > 0x7fffffffull || lo_first >= n || hi_last > n ||
      hi_last == 0 || (nw == 1 && hi_last <= lo_first)) {
    set_error("multiexp: grid share [window %u term %zu, window %u term %zu) outside the %u x %zu grid", w0,
              lo_first, w0 + nw - 1, hi_last, pl.W, n);
    return ECG_ERR_INVALID;
  }
  GridBlocks gb{};
  gb.nb = nw;
  uint64_t off = 0;
  for (uint32_t i = 0; i < nw; i++) {
    const uint64_t lo = i == 0 ? lo_first : 0, hi = i + 1 == nw ? hi_last : n;
    gb.off[i] = off;
    gb.lo[i] = lo;
    gb.len[i] = hi - lo;
    gb.mp[i] = (gb.len[i] + pl.seg - 1) / pl.seg * pl.seg;
    off += gb.mp[i];
  }
  gb.total = off;
  pl.wd = pl.W;
  pl.w0 = w0;
  pl.W = nw;
  pl.G = nw;
  plan_reduction(pl);  // the caller resets the msm_accumulate timer
  MsmGeom g{1, 1, n, n, 0};
  g.grid = &gb;
  void* d_sums;
  ECG_TRY(msm_core_t<C>(ctx, d_bases, d_scalars, g, pl, s, &d_sums, bf.prepared));
  const MsmPlan e = msm_eff_plan<C>(pl);
  X* win;
  ECG_TRY(msm_sums_to_host(ctx, d_sums, msm_single_sums(e), s, &win));
  HX total = HX::zero();
  msm_host_fold_bits<C>(win, e, total);
  host::hto_jac_norm(total, out_jac);
  return ECG_OK;
}

// Terms per device pass: calc_chunk_size (multiexp.rs:71-93) restated for
// this pipeline's workspace.  Per term: the staged input base
// and scalar (host-slice entry points), the reduced-radix base record, W
// double-buffered (key, value) pairs and the segment-edge records (2 per SEG
// entries, + 1/16 for the next combine level); fixed: the W x B buckets and
// the sort's scratch.  MEMORY_PADDING of the device memory and the resident
// base cache are left alone.  ecg_ctx_set_msm_chunk pins the value instead.
template <class C>
double msm_term_bytes(const MsmPlan& pl) {
  using F = typename C::Fq;
  constexpr bool rr = MsmField<C>::rr;
  using AF = typename MsmField<C>::type;
  return 2.0 * sizeof(F) + 32.0 + (rr ? (double)BaseLayout<AF>::BYTES : 0.0) + 16.0 * pl.W +
         2.0 * pl.W / pl.seg * (sizeof(XYZZ<AF>) + 4) * (1.0 + 1.0 / 16);
}

// Device memory left for an MSM's workspace: (1 - MEMORY_PADDING) of the
// context's memory, minus the resident base cache and 256 MB of scratch --
// and never more than the device can still give this context: its free
// memory now plus what the context's MSM buffers already hold (they regrow in
// place), less 2 % of the device for the allocator's granularity.  The second
// bound accounts for what the first cannot see: prepared bases and scalars the
// caller keeps resident (68.7 + 17.2 GB for a 2^29 MSM), other contexts'
// workspaces, other processes.
template <class C>
double msm_mem_budget(const ecg_ctx* ctx) {
  double cached = 0;
  for (const auto& e : ctx->base_cache) cached += (double)e.n * msm_base_record_bytes<C>();  // prepared entries
  const double budget = (double)ctx_mem(ctx) * (1.0 - MSM_MEMORY_PADDING) - cached - 256.0 * (1 << 20);
  size_t dev_free = 0, dev_total = 0;
  if (hipMemGetInfo(&dev_free, &dev_total) != hipSuccess) {
    (void)hipGetLastError();
    return budget;
  }
  double held = 0;
  for (const auto& kv : ctx->ws)
    if (kv.first.compare(0, 4, "msm_") == 0) held += (double)kv.second.bytes;
  const double avail = (double)dev_free + held - 0.02 * (double)dev_total - 256.0 * (1 << 20);
  return avail < budget ? avail : budget;
}

template <class C>
size_t msm_pass_terms(const ecg_ctx* ctx) {
  if (ctx->msm_chunk) return ctx->msm_chunk;
  using AF = typename MsmField<C>::type;
  const MsmPlan pl = make_plan((size_t)1 << 26, (uint32_t)C::FrParams::BITS);
  const double fixed = (double)pl.W * pl.B * sizeof(XYZZ<AF>);  // one bucket array
  double t = (msm_mem_budget<C>(ctx) - fixed) / msm_term_bytes<C>(pl);
  if (!(t >= (double)(1u << 16))) t = (double)(1u << 16);  // tiny / unknown memory: still make progress
  if (t > (double)0x7fffffffu) t = (double)0x7fffffffu;   // 31-bit term indices
  return (size_t)t;
}

// One MSM, processed in device passes of msm_pass_terms terms (the
// reference's sub-chunk loop, multiexp.rs:348-361, with the abort poll before
// each pass, :140-144); the window sums come back to the host, which runs the
// Horner fold of each pass and adds the passes up.
template <class C>
int msm_single_t(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, uint64_t* out_jac,
                        hipStream_t s, ecg_abort_cb abort_cb, void* user, uint32_t scalar_mont, BaseForm bf) {
  const bool prepared = bf.prepared;
  using F = typename C::Fq;
  using X = XYZZ<F>;
  using HX = host::HPoint<HostF<C>>;
  kt_reset(ctx, "msm_accumulate");
  HX total_acc = HX::zero();
  const size_t chunk = msm_pass_terms<C>(ctx);
  for (size_t off = 0; off < n; off += chunk) {
    if (abort_cb && abort_cb(user)) return ECG_ABORTED;  // multiexp.rs:140-144
    const size_t m = n - off < chunk ? n - off : chunk;
    const MsmPlan pl = bf.tab_c ? make_tab_plan(1, (uint32_t)C::FrParams::BITS, bf.tab_c, bf.tab_n)
                                : make_plan(m, (uint32_t)C::FrParams::BITS);
    const MsmGeom g{1, 1, m, m, scalar_mont};
    void* d_sums;
    const void* bp = prepared ? (const void*)((const char*)d_bases + off * msm_base_record_bytes<C>() *
                                              (bf.tab_c ? pl.W : 1u))
                              : (const void*)((const F*)d_bases + 2 * off);
    ECG_TRY(msm_core_t<C>(ctx, bp, (const uint4*)d_scalars + 2 * off, g, pl, s, &d_sums, prepared));
    // window A / offset-bit sums -> host; Horner fold over windows (multiexp.rs:221-233)
    const MsmPlan e = msm_eff_plan<C>(pl);
    const size_t nw = msm_single_sums(e);
    X* win;
    ECG_TRY(msm_sums_to_host(ctx, d_sums, nw, s, &win));
    msm_host_fold_bits<C>(win, e, total_acc);
  }
  host::hto_jac_norm(total_acc, out_jac);
  return ECG_OK;
}


static uint32_t msm_h2d_passes() {  // host-slice pipeline depth (A/B: ECG_MSM_H2D_PASSES)
  static const uint32_t v = env_u32_in("ECG_MSM_H2D_PASSES", 4, 1, 64);
  return v ? v : 1;
}

// MSM over HOST slices -- the reference's own entry (SingleMultiexpKernel::
// multiexp copies bases and exps in on every call, multiexp.rs:152-164).
// Instead of copying all 128 B/term and then computing, the terms run as
// passes whose upload overlaps the previous pass's compute: pass k+1's bases
// and scalars go H2D on a copy stream into the other half of a double-
// buffered staging area while the compute stream runs pass k (the
// accumulation is VALU-bound, the copy is PCIe-bound).  Every pass of a batch
// of up to MSM_MAX_SLOTS passes fills its own bucket slot with one plan for
// the whole MSM, and ONE reduction sums the slots bucket by bucket
// (msm_reduce_kernel adds them into its running sums): a pass costs its
// digits, sort and accumulation, not a reduction of 2^(c-1) W buckets of its
// own.  Same group element as the single-pass MSM.
// bf.prepared: `bases` is a device-resident prepared buffer (the base cache of
// ecg_msm_ex, an Arc<Vec<G>> seen again): only the 32-B scalars travel, and
// the passes grow geometrically (first n / 16, then x2): the first pass's
// upload is the only one not hidden behind compute.
constexpr uint32_t MSM_MAX_SLOTS = 8;
// Bucket slots a pipelined MSM may hold at once: one bucket array per pass of
// a batch (W x B XYZZ buckets each; 1.5 GB for BLS12-381 at c = 20, 5.6 GB at
// c = 22), as many as the memory left after the largest pass's per-term
// workspace allows, at most MSM_MAX_SLOTS.  Passes beyond it form more batches
// (one reduction each).  msm_pass_terms budgets one array only.
template <class C>
uint32_t msm_slot_cap(const ecg_ctx* ctx, const MsmPlan& pl, size_t pmax) {
  using AF = typename MsmField<C>::type;
  const double slot = (double)pl.G * pl.B * sizeof(XYZZ<AF>);
  const double left = msm_mem_budget<C>(ctx) - (double)pmax * msm_term_bytes<C>(pl);
  const double k = left / slot;
  if (!(k >= 1.0)) return 1;
  return k >= MSM_MAX_SLOTS ? MSM_MAX_SLOTS : (uint32_t)k;
}
// fill (a cache miss of ecg_msm_ex, msm_prepared_alloc'd `bases`): the host
// bases of each pass go up with its scalars (104 B ark records or 96 B [x, y])
// and become the buffer's records on the device before the pass reads them;
// the copies dominate (136 B/term against ~2.2 ns of compute per term), so the
// passes are equal, MSM_MAX_SLOTS of them.
template <class C>
int msm_host_t(ecg_ctx* ctx, const void* bases, BaseForm bf, const void* h_scalars, size_t n, uint32_t scalar_mont,
               uint64_t* out_jac, ecg_abort_cb abort_cb, void* user, const MsmFill* fill) {
  using F = typename C::Fq;
  using X = XYZZ<F>;
  using HX = host::HPoint<HostF<C>>;
  kt_reset(ctx, "msm_accumulate");
  if (n == 0) {
    host::hto_jac_norm(HX::zero(), out_jac);
    return ECG_OK;
  }
  const bool resident = bf.prepared;
  const size_t sb = 32;
  // host bytes per base of the pass uploads: [x, y], the fill's layout, or none
  const size_t bb = fill ? (fill->ark ? 2 * sizeof(F) + 8 : 2 * sizeof(F)) : (resident ? 0 : 2 * sizeof(F));
  const void* hb = fill ? fill->h_bases : bases;
  // ---- pass sizes
  const size_t maxpass = msm_pass_terms<C>(ctx);
  std::vector<size_t> poff{0};
  if (fill && n >= ((size_t)1 << 22)) {
    const size_t pass = std::min(maxpass, (n + MSM_MAX_SLOTS - 1) / MSM_MAX_SLOTS);
    for (size_t o = pass; o < n; o += pass) poff.push_back(o);
    poff.push_back(n);
  } else if (n >= ((size_t)1 << 22) && resident && !fill) {
    // A/B: ECG_MSM_PASS_FIRST (1/x of n) and ECG_MSM_PASS_GROWTH
    static const uint32_t first_div = env_u32_in("ECG_MSM_PASS_FIRST", 16, 1, 1024);
    static const uint32_t growth = env_u32_in("ECG_MSM_PASS_GROWTH", 3, 2, 16);
    size_t m = std::max<size_t>((n / first_div + 255) / 256 * 256, 1);
    while (poff.back() < n) {
      const size_t left = n - poff.back();
      const size_t take = std::min({m, left, maxpass});
      poff.push_back(poff.back() + (left - take < m / 2 && left <= maxpass ? left : take));  // no tiny last pass
      m *= growth;
    }
  } else {
    size_t pass = maxpass;
    if (n >= ((size_t)1 << 22)) pass = std::min(pass, (n + msm_h2d_passes() - 1) / msm_h2d_passes());
    for (size_t o = pass; o < n; o += pass) poff.push_back(o);
    poff.push_back(n);
  }
  const size_t np = poff.size() - 1;
  size_t pmax = 0;
  for (size_t k = 0; k < np; k++) pmax = std::max(pmax, poff[k + 1] - poff[k]);
  // one plan for every pass: passes of a batch share its bucket slots
  const MsmPlan pl = bf.tab_c ? make_tab_plan(1, (uint32_t)C::FrParams::BITS, bf.tab_c, bf.tab_n)
                              : make_plan(n, (uint32_t)C::FrParams::BITS);
  const size_t nsums = msm_single_sums(msm_eff_plan<C>(pl));
  const uint32_t slot_cap = msm_slot_cap<C>(ctx, pl, pmax);
  const size_t nbatch = (np + slot_cap - 1) / slot_cap;
  const uint32_t slots = (uint32_t)std::min<size_t>(np, slot_cap);
  // bytes per base of the resident buffer (all of its table rows)
  const size_t rstride = msm_base_record_bytes<C>() * (bf.tab_c ? msm_table_windows<C>(bf.tab_c) : 1u);
  void *ib[2] = {nullptr, nullptr}, *is[2] = {nullptr, nullptr}, *sums, *fxy = nullptr;
  if (bb) ECG_TRY(ws_get(ctx, "msm_in_bases", pmax * bb, &ib[0]));
  ECG_TRY(ws_get(ctx, "msm_in_scalars", pmax * sb, &is[0]));
  if (np > 1) {
    if (bb) ECG_TRY(ws_get(ctx, "msm_in_bases_b", pmax * bb, &ib[1]));
    ECG_TRY(ws_get(ctx, "msm_in_scalars_b", pmax * sb, &is[1]));
  }
  if (fill && fill->ark) ECG_TRY(ws_get(ctx, "msm_fill_xy", pmax * 2 * sizeof(F), &fxy));
  ECG_TRY(ws_get(ctx, "msm_pass_sums", nbatch * nsums * sizeof(X), &sums));
  if (!ctx->copy_stream) ECG_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  hipStream_t cs = ctx->stream, us = ctx->copy_stream;
  {  // every workspace buffer at its largest size before the pipeline starts
    const MsmGeom g{1, 1, pmax, pmax, scalar_mont};
    void* unused = nullptr;
    ECG_TRY(msm_core_t<C>(ctx, bases, is[0], g, pl, cs, &unused, resident, nullptr, CORE_RESERVE,
                          MsmSlots{0, slots}));
  }
  hipEvent_t up[2], done[2];
  for (int i = 0; i < 2; i++) {
    ECG_HIP(hipEventCreateWithFlags(&up[i], hipEventDisableTiming));
    ECG_HIP(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
  }
  auto upload = [&](size_t k) -> int {
    const size_t off = poff[k], m = poff[k + 1] - off;
    const int b = (int)(k & 1);
    if (bb) ECG_HIP(hipMemcpyAsync(ib[b], (const uint8_t*)hb + off * bb, m * bb, hipMemcpyHostToDevice, us));
    ECG_HIP(hipMemcpyAsync(is[b], (const uint8_t*)h_scalars + off * sb, m * sb, hipMemcpyHostToDevice, us));
    ECG_HIP(hipEventRecord(up[b], us));
    return ECG_OK;
  };
  int rc = upload(0);
  for (size_t k = 0; rc == ECG_OK && k < np; k++) {
    if (abort_cb && abort_cb(user)) {  // multiexp.rs:140-144, before every pass
      rc = ECG_ABORTED;
      break;
    }
    const int b = (int)(k & 1);
    const size_t m = poff[k + 1] - poff[k];
    const MsmGeom g{1, 1, m, m, scalar_mont};
    const size_t batch = k / slot_cap;
    const uint32_t slot = (uint32_t)(k % slot_cap);
    const bool last_of_batch = slot + 1 == slot_cap || k + 1 == np;
    const void* bp = resident ? (const void*)((const uint8_t*)bases + poff[k] * rstride) : ib[b];
    rc = [&]() -> int {
      ECG_HIP(hipStreamWaitEvent(cs, up[b], 0));
      if (fill) {  // this pass's records of the cache entry, from the uploaded host bases
        const void* xy = ib[b];
        if (fill->ark) {
          ECG_TRY(bases_from_ark(ctx, fill->curve_id, ib[b], m, fxy, cs));
          xy = fxy;
        }
        ECG_TRY(msm_records_t<C>(xy, m, const_cast<void*>(bp), cs));
      }
      void* d_sums = nullptr;
      ECG_TRY(msm_core_t<C>(ctx, bp, is[b], g, pl, cs, &d_sums, resident, nullptr, CORE_ACC, MsmSlots{slot, slots}));
      ECG_HIP(hipEventRecord(done[b], cs));
      if (k + 1 < np) {
        if (k >= 1) ECG_HIP(hipStreamWaitEvent(us, done[b ^ 1], 0));  // pass k-1 has released its staging half
        ECG_TRY(upload(k + 1));
      }
      if (last_of_batch) {  // one reduction over the batch's slots
        ECG_TRY(msm_core_t<C>(ctx, bp, is[b], g, pl, cs, &d_sums, resident, nullptr, CORE_FIN,
                              MsmSlots{0, slot + 1}));
        ECG_HIP(hipMemcpyAsync((X*)sums + batch * nsums, d_sums, nsums * sizeof(X), hipMemcpyDefault, cs));
      }
      return ECG_OK;
    }();
  }
  (void)hipStreamSynchronize(us);
  X* win = nullptr;
  if (rc == ECG_OK) {
    rc = [&]() -> int {
      ECG_TRY(hws_get(ctx, "msm_win", nbatch * nsums * sizeof(X), (void**)&win));  // pinned
      ECG_HIP(hipMemcpyAsync(win, sums, nbatch * nsums * sizeof(X), hipMemcpyDeviceToHost, cs));
      ECG_HIP(hipStreamSynchronize(cs));
      return ECG_OK;
    }();
  } else {
    (void)hipStreamSynchronize(cs);
  }
  for (int i = 0; i < 2; i++) {
    (void)hipEventDestroy(up[i]);
    (void)hipEventDestroy(done[i]);
  }
  if (rc != ECG_OK) return rc;
  HX total = HX::zero();
  const MsmPlan e = msm_eff_plan<C>(pl);
  for (size_t k = 0; k < nbatch; k++) msm_host_fold_bits<C>(win + k * nsums, e, total);
  host::hto_jac_norm(total, out_jac);
  return ECG_OK;
}

// Batched multi-line MSM (ag-cuda-ec multiple_multiexp): all tasks in one
// pass -- one sort over (task, window, bucket) keys, one accumulation launch,
// one reduction -- then a device fold per task.  out_jac: tasks x 3 x Fq,
// line-major (results[line * n_chunks + chunk], multiexp.cl:260).
// Batched results normalised on the host (one batch inversion) up to this many
// tasks; more tasks keep the device's thread-per-task normalisation, whose
// latency does not grow with the task count.
constexpr uint32_t MSM_HOST_NORM_TASKS = 2048;
template <class C>
int msm_batch_t(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, const MsmGeom& g,
                       uint32_t window_bits, uint64_t* out_jac, hipStream_t s, BaseForm bf) {
  using F = typename C::Fq;
  const bool prepared = bf.prepared;
  kt_reset(ctx, "msm_accumulate");
  const uint32_t tasks = g.tasks();
  const size_t ob = (size_t)tasks * 3 * sizeof(F);
  if (g.clen == 0) {  // empty chunks: every task is the identity
    using HX = host::HPoint<HostF<C>>;
    for (uint32_t t = 0; t < tasks; t++) host::hto_jac_norm(HX::zero(), out_jac + (size_t)t * 3 * HostF<C>::N);
    return ECG_OK;
  }
  MsmPlan pl;
  if (bf.tab_c) {  // the table fixes the window (window_size is a tuning hint, results never depend on it)
    pl = make_tab_plan(tasks, (uint32_t)C::FrParams::BITS, bf.tab_c, bf.tab_n);
  } else {
    pl = make_plan(g.clen, (uint32_t)C::FrParams::BITS, window_bits);
    pl.G = tasks * pl.W;
    plan_reduction(pl);
  }
  if ((uint64_t)pl.G * pl.B >= 0xffffffffull) {
    set_error("multiple_multiexp: %u tasks x %u windows x %u buckets exceeds the 32-bit bucket space", tasks, pl.W,
              pl.B);
    return ECG_ERR_INVALID;
  }
  void *d_sums, *d_out;
  bool folded = false;
  ECG_TRY(msm_core_t<C>(ctx, d_bases, d_scalars, g, pl, s, &d_sums, prepared, &folded));
  ECG_TRY(ws_get(ctx, "msm_batch_out", ob, &d_out));
  if (folded && tasks <= MSM_HOST_NORM_TASKS) {
    // normalisation on the host with one inversion for all tasks (Montgomery's
    // trick): a device thread per task would wait out a ~380-squaring Fermat
    // chain of its own
    using HF = HostF<C>;
    using HX = host::HPoint<HF>;
    XYZZ<F>* sums;  // pinned staging
    ECG_TRY(hws_get(ctx, "msm_task_sums", (size_t)tasks * sizeof(XYZZ<F>), (void**)&sums));
    ECG_HIP(hipMemcpyAsync(sums, d_sums, (size_t)tasks * sizeof(XYZZ<F>), hipMemcpyDeviceToHost, s));
    ECG_HIP(hipStreamSynchronize(s));
    std::vector<HX> pts(tasks);
    std::vector<HF> pre(tasks);
    HF run = HF::one();
    for (uint32_t t = 0; t < tasks; t++) {
      static_assert(sizeof(pts[t].X) == sizeof(sums[t].X), "host/device coordinate layouts differ");
      memcpy(&pts[t].X, &sums[t].X, sizeof(pts[t].X));
      memcpy(&pts[t].Y, &sums[t].Y, sizeof(pts[t].Y));
      memcpy(&pts[t].ZZ, &sums[t].ZZ, sizeof(pts[t].ZZ));
      memcpy(&pts[t].ZZZ, &sums[t].ZZZ, sizeof(pts[t].ZZZ));
      pts[t].X = host::hcanon(pts[t].X);  // device values are in the lazy range [0, 2p]
      pts[t].Y = host::hcanon(pts[t].Y);
      pts[t].ZZ = host::hcanon(pts[t].ZZ);
      pts[t].ZZZ = host::hcanon(pts[t].ZZZ);
      pre[t] = run;  // product of the (ZZ ZZZ) of the non-identity points before t
      if (!pts[t].is_zero()) run = host::hmul(run, host::hmul(pts[t].ZZ, pts[t].ZZZ));
    }
    HF inv = host::hinv(run);  // 1 / prod (ZZ ZZZ)
    constexpr int N = HF::N;
    for (int t = (int)tasks - 1; t >= 0; t--) {
      uint64_t* o = out_jac + (size_t)t * 3 * N;
      if (pts[t].is_zero()) {
        host::hto_jac_norm(pts[t], o);
        continue;
      }
      const HF d = host::hmul(pts[t].ZZ, pts[t].ZZZ);
      const HF it = host::hmul(inv, pre[t]);  // 1 / (ZZ ZZZ) of point t
      inv = host::hmul(inv, d);
      const HF x = host::hmul(pts[t].X, host::hmul(it, pts[t].ZZZ));
      const HF y = host::hmul(pts[t].Y, host::hmul(it, pts[t].ZZ));
      const HF one = HF::one();
      memcpy(o, &x, 8 * N);
      memcpy(o + N, &y, 8 * N);
      memcpy(o + 2 * N, &one, 8 * N);
    }
    return ECG_OK;
  }
  MsmPlan pf = pl;
  if (folded) pf.tab = 1;  // one (already folded) sum per task: normalisation only
  hipLaunchKernelGGL(msm_fold_kernel<C>, dim3(blocks_for(tasks, 64)), dim3(64), 0, s, (const XYZZ<F>*)d_sums, pf,
                     tasks, (F*)d_out);
  ECG_HIP(hipGetLastError());
  void* h_out;  // pinned staging, then the caller's buffer
  ECG_TRY(hws_get(ctx, "msm_batch_out", ob, &h_out));
  ECG_HIP(hipMemcpyAsync(h_out, d_out, ob, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  memcpy(out_jac, h_out, ob);
  return ECG_OK;
}


template <class C>
int point_sum_host_t(const uint64_t* pts, size_t count, uint64_t* out_jac) {
  using HF = HostF<C>;
  host::HPoint<HF> acc = host::HPoint<HF>::zero();
  for (size_t i = 0; i < count; i++) acc = host::hadd_pts(acc, host::hfrom_jac_t<HF>(&pts[i * 3 * HF::N]));
  host::hto_jac_norm(acc, out_jac);
  return ECG_OK;
}



template <class C>
int gen_bases_t(ecg_ctx* ctx, const uint64_t* a, const uint64_t* b, size_t n, void* d_out, hipStream_t s) {
  using F = typename C::Fq;
  using S = Fp<typename C::FrParams>;
  if (n == 0) return ECG_OK;
  // a, b arrive canonical; the kernels convert to Montgomery themselves.
  S ac, bc;
  memcpy(ac.v, a, sizeof(ac.v));
  memcpy(bc.v, b, sizeof(bc.v));
  void *q, *scratch;
  ECG_TRY(ws_get(ctx, "gen_q", 2 * sizeof(F), &q));
  ECG_TRY(ws_get(ctx, "gen_scratch", n * 3 * sizeof(F), &scratch));
  hipLaunchKernelGGL(gen_step_kernel<C>, dim3(1), dim3(64), 0, s, bc, (F*)q);
  ECG_HIP(hipGetLastError());
  const size_t threads = (n + GEN_BLOCK - 1) / GEN_BLOCK;
  hipLaunchKernelGGL(gen_bases_kernel<C>, dim3(blocks_for(threads, MSM_THREADS)), dim3(MSM_THREADS), 0, s,
                     ac, bc, n, (const F*)q, (F*)d_out, (F*)scratch);
  ECG_HIP(hipGetLastError());
  ECG_HIP(hipStreamSynchronize(s));
  ws_release(ctx, "gen_scratch");
  return ECG_OK;
}


}  // namespace ecg
