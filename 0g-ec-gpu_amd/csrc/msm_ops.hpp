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
};

}  // namespace ecg
