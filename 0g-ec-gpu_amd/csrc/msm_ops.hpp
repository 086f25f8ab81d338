// Per-curve MSM entry points (msm_inst.hip), routed by msm.hip.
#pragma once
#include "ctx.hpp"

namespace ecg {

struct MsmOps {
  int (*single)(ecg_ctx*, const void* d_bases, const void* d_scalars, size_t n, uint64_t* out_jac, hipStream_t,
                ecg_abort_cb, void* user, uint32_t scalar_mont, BaseForm bf);
  int (*batch)(ecg_ctx*, const void* d_bases, const void* d_scalars, uint32_t n_lines, uint32_t n_chunks,
               size_t line_len, uint32_t scalar_mont, uint32_t window_bits, uint64_t* out_jac, hipStream_t,
               BaseForm bf);
  // bases [x, y] -> the bucket kernels' layout (prepared_bytes(n, tab_c) bytes at d_out); tab_c > 0 builds
  // the window table (G1 only)
  int (*prepare)(ecg_ctx*, const void* d_bases, size_t n, uint32_t tab_c, void* d_out, hipStream_t);
  size_t (*prepared_bytes)(size_t n, uint32_t tab_c);
  uint32_t (*table_windows)(uint32_t tab_c);  // rows of a window table (0: no table form for this curve)
  uint32_t (*table_auto)(size_t n);           // window size of an automatic table for n-term MSMs
  int (*point_sum)(const uint64_t* points, size_t count, uint64_t* out_jac);
  int (*gen_bases)(ecg_ctx*, const uint64_t* a, const uint64_t* b, size_t n, void* d_out, hipStream_t);
  size_t (*pass_terms)(const ecg_ctx*);
  // host scalars, pipelined with compute; bases on the host ([x, y]), or with
  // bf.prepared a device-resident prepared buffer
  int (*host)(ecg_ctx*, const void* bases, BaseForm bf, const void* h_scalars, size_t n, uint32_t scalar_mont,
              uint64_t* out_jac, ecg_abort_cb, void* user, const MsmFill* fill);
  size_t (*record_bytes)();  // bytes per prepared base record (one table row)
  int (*plan_info)(size_t n, uint32_t window_bits, uint32_t* c, uint32_t* windows, int* sort_mode);
  // windows [w0, w0 + nwin) of the n_plan-term plan over m terms (msm_piece_t)
  int (*piece)(ecg_ctx*, const void* d_bases, const void* d_scalars, size_t m, size_t n_plan, uint32_t w0,
               uint32_t nwin, uint64_t* out_jac, hipStream_t, BaseForm bf);
  // a rank's whole grid share in one core call (msm_grid_t)
  int (*grid)(ecg_ctx*, const void* d_bases, const void* d_scalars, size_t n, uint32_t w0, uint32_t nw,
              size_t lo_first, size_t hi_last, uint64_t* out_jac, hipStream_t, BaseForm bf);
};

// This rank's share of an n-term MSM split over a grid of (window x term)
// ranges (ecg_msm_dist_grid): the W windows of the n-term plan times the n
// terms, in window-major order, cut into nranks equal contiguous ranges; rank
// `rank` runs its range's pieces (a partial window, whole windows, a partial
// window) over the full base and scalar arrays and returns their partial sum.
// *pieces receives the number of pieces run.
int msm_grid_run(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n, int rank,
                 int nranks, uint64_t* out_jac, hipStream_t s, ecg_abort_cb abort_cb, void* user, int* pieces);

}  // namespace ecg
