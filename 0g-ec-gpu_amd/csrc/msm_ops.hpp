// Per-curve MSM entry points (msm_inst.hip), routed by msm.hip.
#pragma once
#include "ctx.hpp"

namespace ecg {

struct MsmOps {
  int (*single)(ecg_ctx*, const void* d_bases, const void* d_scalars, size_t n, uint64_t* out_jac, hipStream_t,
                ecg_abort_cb, void* user, uint32_t scalar_mont);
  int (*batch)(ecg_ctx*, const void* d_bases, const void* d_scalars, uint32_t n_lines, uint32_t n_chunks,
               size_t line_len, uint32_t scalar_mont, uint32_t window_bits, uint64_t* out_jac, hipStream_t);
  int (*point_sum)(const uint64_t* points, size_t count, uint64_t* out_jac);
  int (*gen_bases)(ecg_ctx*, const uint64_t* a, const uint64_t* b, size_t n, void* d_out, hipStream_t);
  size_t (*pass_terms)(const ecg_ctx*);
  int (*host)(ecg_ctx*, const void* h_bases, const void* h_scalars, size_t n, uint64_t* out_jac, ecg_abort_cb,
              void* user);
};

}  // namespace ecg
