// One curve's MSM kernels and drivers (msm_impl.hpp), compiled once per curve
// with -DECG_INST=<curve id> so the four instantiations build in parallel.
#include "msm_impl.hpp"
#include "msm_ops.hpp"

#ifndef ECG_INST
#error "compile with -DECG_INST=<curve id>"
#endif

namespace ecg {

#if ECG_INST == 0
using InstCurve = BLS12_381;
#define ECG_OPS_NAME msm_ops_0
#elif ECG_INST == 1
using InstCurve = BN254;
#define ECG_OPS_NAME msm_ops_1
#elif ECG_INST == 2
using InstCurve = BLS12_381_G2;
#define ECG_OPS_NAME msm_ops_2
#else
using InstCurve = BN254_G2;
#define ECG_OPS_NAME msm_ops_3
#endif

static int batch_entry(ecg_ctx* ctx, const void* d_bases, const void* d_scalars, uint32_t n_lines, uint32_t n_chunks,
                       size_t line_len, uint32_t scalar_mont, uint32_t window_bits, uint64_t* out_jac,
                       hipStream_t s, BaseForm bf) {
  const MsmGeom g{n_lines, n_chunks, line_len, line_len / n_chunks, scalar_mont};
  return msm_batch_t<InstCurve>(ctx, d_bases, d_scalars, g, window_bits, out_jac, s, bf);
}

extern MsmOps ECG_OPS_NAME;
MsmOps ECG_OPS_NAME = {&msm_single_t<InstCurve>,        &batch_entry,
                       &msm_prepare_t<InstCurve>,       &msm_prepared_bytes<InstCurve>,
                       &msm_table_windows<InstCurve>,   &msm_table_auto<InstCurve>,
                       &point_sum_host_t<InstCurve>,    &gen_bases_t<InstCurve>,
                       &msm_pass_terms<InstCurve>,      &msm_host_t<InstCurve>,
                       &msm_base_record_bytes<InstCurve>, &msm_plan_info_t<InstCurve>,
                       &msm_piece_t<InstCurve>,
                       &msm_grid_t<InstCurve>};

}  // namespace ecg
