// curve_id dispatch of the MSM drivers.  The per-curve kernels and drivers
// (msm_impl.hpp) are compiled once per curve in msm_inst.hip (-DECG_INST=id),
// which exports one MsmOps table each; this file only routes calls.
#include <vector>

#include "ctx.hpp"
#include "msm_ops.hpp"

namespace ecg {

extern MsmOps msm_ops_0, msm_ops_1, msm_ops_2, msm_ops_3;

static const MsmOps* msm_ops(int curve_id, const char* what) {
  switch (curve_id) {
    case ECG_CURVE_BLS12_381: return &msm_ops_0;
    case ECG_CURVE_BN254: return &msm_ops_1;
    case ECG_CURVE_BLS12_381_G2: return &msm_ops_2;
    case ECG_CURVE_BN254_G2: return &msm_ops_3;
    default:
      set_error("%s: unknown curve_id %d", what, curve_id);
      return nullptr;
  }
}

// Is d_bases a prepared buffer (ecg_msm_prepare_bases / _table)?  It must
// then cover the n bases the call reads, for the same curve.
static int prepared_lookup(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n, const char* what,
                           BaseForm* bf) {
  *bf = BaseForm{};
  auto it = ctx->prepared.find(d_bases);
  if (it == ctx->prepared.end()) return ECG_OK;
  if (it->second.curve != curve_id || n > it->second.n) {
    set_error("%s: prepared bases are %zu bases of curve %d, the call reads %zu of curve %d", what, it->second.n,
              it->second.curve, n, curve_id);
    return ECG_ERR_INVALID;
  }
  bf->prepared = true;
  bf->tab_c = it->second.tab_c;
  bf->tab_n = it->second.n;
  return ECG_OK;
}

int msm_run(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n, uint64_t* out_jac,
            hipStream_t s, ecg_abort_cb abort_cb, void* user, int scalar_mont) {
  if (n > 0x7fffffffull) {
    set_error("multiexp: at most 2^31-1 terms per call");
    return ECG_ERR_INVALID;
  }
  const MsmOps* o = msm_ops(curve_id, "multiexp");
  if (!o) return ECG_ERR_INVALID;
  BaseForm bf;
  ECG_TRY(prepared_lookup(ctx, curve_id, d_bases, n, "multiexp", &bf));
  return o->single(ctx, d_bases, d_scalars, n, out_jac, s, abort_cb, user, scalar_mont != 0, bf);
}

uint32_t msm_table_window_auto(int curve_id, size_t n) {
  const MsmOps* o = msm_ops(curve_id, "prepare_table");
  return o ? o->table_auto(n) : 0;
}

int msm_prepare_run(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n, uint32_t tab_c, void** d_out,
                    hipStream_t s) {
  const MsmOps* o = msm_ops(curve_id, "prepare_bases");
  if (!o) return ECG_ERR_INVALID;
  if (tab_c) {
    if (tab_c < 2 || tab_c > 25) {
      set_error("prepare_table: window size %u out of range [2, 25]", tab_c);
      return ECG_ERR_INVALID;
    }
    const uint32_t W = o->table_windows(tab_c);
    if (!W) {
      set_error("prepare_table: window tables are built for the G1 curves only (curve %d)", curve_id);
      return ECG_ERR_INVALID;
    }
    if ((uint64_t)W * n >= 0x80000000ull) {
      set_error("prepare_table: %u rows x %zu bases exceeds the 2^31 table-index space", W, n);
      return ECG_ERR_INVALID;
    }
  }
  const size_t bytes = o->prepared_bytes(n, tab_c);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("prepare_bases: device allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return ECG_ERR_NOMEM;
  }
  int rc = o->prepare(ctx, d_bases, n, tab_c, p, s);
  if (rc == ECG_OK && hipStreamSynchronize(s) != hipSuccess) {
    set_error("prepare_bases: %s", hipGetErrorString(hipGetLastError()));
    rc = ECG_ERR_HIP;
  }
  if (rc != ECG_OK) {
    (void)hipFree(p);
    return rc;
  }
  ctx->prepared[p] = {curve_id, n, tab_c};
  *d_out = p;
  return ECG_OK;
}

int msm_batch_run(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n_bases, const void* d_scalars,
                  int scalar_mont, size_t line_len, size_t n_chunks, uint32_t window_bits, uint64_t* out_jac,
                  hipStream_t s) {
  if (line_len == 0 || n_chunks == 0) {
    set_error("multiple_multiexp: line_len and num_chunks must be positive");
    return ECG_ERR_INVALID;
  }
  if (n_bases % line_len != 0) {
    set_error("multiple_multiexp: %zu bases is not a whole number of lines of %zu", n_bases, line_len);
    return ECG_ERR_INVALID;
  }
  if (n_bases > 0x7fffffffull) {
    set_error("multiple_multiexp: at most 2^31-1 bases per call");
    return ECG_ERR_INVALID;
  }
  if (window_bits > 22) {
    set_error("multiple_multiexp: window_size %u out of range [0, 22] (0 = automatic)", window_bits);
    return ECG_ERR_INVALID;
  }
  const size_t n_lines = n_bases / line_len;
  if (n_lines == 0) return ECG_OK;
  if (n_lines * n_chunks > 0xffffffull) {
    set_error("multiple_multiexp: %zu tasks is too many", n_lines * n_chunks);
    return ECG_ERR_INVALID;
  }
  const MsmOps* o = msm_ops(curve_id, "multiple_multiexp");
  if (!o) return ECG_ERR_INVALID;
  BaseForm bf;
  ECG_TRY(prepared_lookup(ctx, curve_id, d_bases, n_bases, "multiple_multiexp", &bf));
  return o->batch(ctx, d_bases, d_scalars, (uint32_t)n_lines, (uint32_t)n_chunks, line_len, scalar_mont != 0,
                  window_bits, out_jac, s, bf);
}

int point_sum_host(int curve_id, const uint64_t* points, size_t count, uint64_t* out_jac) {
  const MsmOps* o = msm_ops(curve_id, "point_sum");
  if (!o) return ECG_ERR_INVALID;
  return o->point_sum(points, count, out_jac);
}

int point_sum_run(ecg_ctx* ctx, int curve_id, const void* d_points, size_t count, uint64_t* out_jac, hipStream_t s) {
  if (!curve_valid(curve_id)) {
    set_error("point_sum: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  std::vector<uint64_t> pts(count * 3 * (size_t)fq_limbs64(curve_id));
  if (count) ECG_HIP(hipMemcpyAsync(pts.data(), d_points, pts.size() * 8, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  (void)ctx;
  return point_sum_host(curve_id, pts.data(), count, out_jac);
}

int msm_host_run(ecg_ctx* ctx, int curve_id, const void* h_bases, const void* h_scalars, size_t n, uint64_t* out_jac,
                 ecg_abort_cb abort_cb, void* user) {
  if (n > 0x7fffffffull) {
    set_error("multiexp: at most 2^31-1 terms per call");
    return ECG_ERR_INVALID;
  }
  const MsmOps* o = msm_ops(curve_id, "multiexp");
  if (!o) return ECG_ERR_INVALID;
  return o->host(ctx, h_bases, h_scalars, n, out_jac, abort_cb, user);
}

int msm_pass_terms_run(const ecg_ctx* ctx, int curve_id, size_t* out) {
  const MsmOps* o = msm_ops(curve_id, "multiexp");
  if (!o) return ECG_ERR_INVALID;
  *out = o->pass_terms(ctx);
  return ECG_OK;
}

int gen_bases_run(ecg_ctx* ctx, int curve_id, const uint64_t* a, const uint64_t* b, size_t n, void* d_out,
                  hipStream_t s) {
  const MsmOps* o = msm_ops(curve_id, "gen_bases");
  if (!o) return ECG_ERR_INVALID;
  return o->gen_bases(ctx, a, b, n, d_out, s);
}

}  // namespace ecg
