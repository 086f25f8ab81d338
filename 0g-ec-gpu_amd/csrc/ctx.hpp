// Internal runtime: device context, grow-only HBM workspace, error state and
// per-kernel HIP-event timing.  Replaces the reference's per-call
// Program::run closures (rust-gpu-tools) and ag-cuda-proxy's CudaWorkspace
// (ag-cuda-proxy/src/module.rs:23-42): here one context = one device + one
// stream + buffers that persist across calls (sized for 288 GB of HBM3E, so
// 2^26-point MSMs and 2^24-point NTTs run as single chunks).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ecgpu.h"

namespace ecg {

void set_error(const char* fmt, ...);

#define ECG_HIP(call)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::ecg::set_error("HIP error %s (%s) at %s:%d", hipGetErrorName(e_),              \
                       hipGetErrorString(e_), __FILE__, __LINE__);                      \
      return ECG_ERR_HIP;                                                               \
    }                                                                                   \
  } while (0)

#define ECG_TRY(expr)          \
  do {                         \
    int rc_ = (expr);          \
    if (rc_ != ECG_OK) return rc_; \
  } while (0)

// Entry of every API call on a context: make its device current and hold the
// context's lock for the rest of the call (one context may be shared by
// several host threads -- e.g. listed twice in ecg_msm_multi's ctxs -- so its
// stream, workspace map and event pool are never used concurrently).
#define ECG_ENTER(ctx)                                   \
  ECG_TRY(::ecg::ctx_enter(ctx));                        \
  std::lock_guard<std::recursive_mutex> ecg_ctx_lock_((ctx)->mu)

struct KernelTimes {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double ms = 0.0;
  int launches = 0;
};

}  // namespace ecg

struct ecg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // H2D staging of the host-slice MSM (lazily created)
  std::recursive_mutex mu;  // held by every API call on this context (ECG_ENTER)
  size_t mem_bytes = 0;
  int compute_units = 0;
  struct Buf {
    void* ptr = nullptr;
    size_t bytes = 0;
  };
  std::map<std::string, Buf> ws;
  // pinned host staging (hws_get): the small D2H copies of results (window
  // sums, task sums) -- a pageable destination cost ~0.2-0.26 ms of host-side
  // staging per MSM before the copy started (profiles/r04/msm_2p2*_timeline.txt)
  std::map<std::string, Buf> hws;
  // FFT twiddle-table cache key
  int tw_fid = -1;
  int tw_variant = 0;
  int tw_full = 0;
  uint32_t tw_log_n = 0;
  uint64_t tw_omega[4] = {0, 0, 0, 0};
  // persistent base cache: converted [x, y] bases keyed by the
  // caller's host buffer, reused while the same (pointer, size, curve,
  // layout) comes back -- the reference's Arc<Vec<G>> bases are immutable.
  struct BaseCache {
    const void* host = nullptr;
    size_t n = 0;
    int curve = -1;
    int layout = -1;
    void* dev = nullptr;
    uint64_t fingerprint = 0;  // sampled host records at upload time
  };
  std::vector<BaseCache> base_cache;
  // (prepared bases -- ecg_msm_prepare_bases -- live in a process-wide
  // registry keyed by device and address range, msm.hip, so any context on
  // the device and any base-aligned pointer into them are recognised)
  // MSM terms per device pass (SingleMultiexpKernel::n, multiexp.rs:71-93);
  // 0 = derived from device memory (msm_chunk_terms)
  size_t msm_chunk = 0;
  // RCCL communicator of this rank (comm.cpp); size 1 / null = single GPU.
  // A host transport (ecg_comm_init_host) replaces it when xchg is set.
  // comm_size > 1 with neither = a communicator aborted after a failure.
  void* comm = nullptr;
  int comm_size = 1;
  int comm_rank = 0;
  ecg_xchg_cb xchg = nullptr;
  void* xchg_user = nullptr;
  uint32_t comm_timeout_ms = 0;  // 0 = ECG_COMM_TIMEOUT_S or the default
  // device staging of the status records (comm.cpp comm_exchange_rec),
  // reserved when an RCCL communicator is set up so that a rank whose call
  // failed on an allocation still joins the status exchange
  void* comm_rec = nullptr;
  size_t comm_rec_bytes = 0;
  // wall time of the last distributed MSM's status + partial exchange
  double comm_last_xchg_us = 0.0;
  // workspace cap (ecg_ctx_set_mem_limit; 0 = the device's memory)
  size_t mem_limit = 0;
  // kernel timing (HIP events on the launch stream)
  std::map<std::string, ecg::KernelTimes> ktimes;
  std::vector<hipEvent_t> event_pool;
};

namespace ecg {

// Make ctx's device current for this host thread.
int ctx_enter(ecg_ctx* ctx);
// Device memory this context plans with: the device's, or its
// ecg_ctx_set_mem_limit cap when that is lower.
inline size_t ctx_mem(const ecg_ctx* ctx) {
  return ctx->mem_limit && ctx->mem_limit < ctx->mem_bytes ? ctx->mem_limit : ctx->mem_bytes;
}
// Grow-only named device buffer.
int ws_get(ecg_ctx* ctx, const char* name, size_t bytes, void** out);
void ws_release(ecg_ctx* ctx, const char* name);
// Grow-only named pinned host buffer (hipHostMalloc, mapped: kernels may write
// it directly through *dev), freed with the context.
int hws_get(ecg_ctx* ctx, const char* name, size_t bytes, void** out, void** dev = nullptr);

// HIP-event bracket for one launch of a named kernel.
hipEvent_t ev_take(ecg_ctx* ctx);
void kt_reset(ecg_ctx* ctx, const char* name);
int kt_begin(ecg_ctx* ctx, const char* name, hipStream_t s);
int kt_end(ecg_ctx* ctx, const char* name, hipStream_t s);
int kt_collect(ecg_ctx* ctx);  // after stream sync

inline hipStream_t pick_stream(ecg_ctx* ctx, void* s) {
  return s ? reinterpret_cast<hipStream_t>(s) : ctx->stream;
}

// Engine entry points (ntt.hip / msm.hip); data pointers are device memory.
int ntt_validate(int field_id, uint32_t log_n);
// batch: that many same-size transforms with the same omega, back to back at d_data
int ntt_run(ecg_ctx* ctx, int field_id, void* d_data, const uint64_t* omega, uint32_t log_n,
            hipStream_t s, ecg_abort_cb abort_cb, void* user, uint32_t batch = 1);
// MSM / point-sum results are written to HOST memory (3 x Lq u64, normalised
// Jacobian): the last serial steps (window fold, normalisation) run on the host.
// scalar_mont: scalars are Montgomery Fr elements (converted on device).
int msm_run(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n,
            uint64_t* out_jac, hipStream_t s, ecg_abort_cb abort_cb, void* user, int scalar_mont = 0);
// Host-side prep moved on device (prep.hip): density compaction of exps
// (DensityTracker::generate_exps), ark Affine{x,y,infinity} -> [x,y].
int density_compact(ecg_ctx* ctx, const void* d_exps, const uint64_t* d_bits, size_t n, void* d_out,
                    size_t* out_count, hipStream_t s);
int bases_from_ark(ecg_ctx* ctx, int curve_id, const void* d_ark, size_t n, void* d_xy, hipStream_t s);
int point_sum_run(ecg_ctx* ctx, int curve_id, const void* d_points, size_t count, uint64_t* out_jac,
                  hipStream_t s);
int ecfft_validate(int curve_id, uint32_t log_n);
int ecfft_run(ecg_ctx* ctx, int curve_id, void* d_jac, const uint64_t* omega, uint32_t log_n, hipStream_t s,
              ecg_abort_cb abort_cb, void* user, uint32_t batch = 1);
// distributed NTT (dfft.hip) and RCCL exchange (comm.cpp)
int dfft_stage1(int field_id, const void* d_in, void* d_out, const uint64_t* omega, uint32_t T, uint32_t rank,
                uint32_t log_n, hipStream_t s);
int dfft_stage3(const void* d_in, void* d_out, uint32_t T, uint32_t log_n, hipStream_t s);
int dfft_run(ecg_ctx* ctx, int field_id, void* d_local, const uint64_t* omega, uint32_t log_n, hipStream_t s,
             ecg_abort_cb abort_cb, void* user);
const char* last_error_text();  // this thread's last error message
int comm_alltoall(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes_per_peer, hipStream_t s);
void comm_free(ecg_ctx* ctx);
int comm_allgather(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes, hipStream_t s);
// Wait for s (collectives included) under the communicator's deadline; on a
// timeout or a collective error the communicator is aborted.
int comm_wait(ecg_ctx* ctx, hipStream_t s, const char* what);
// Every rank's local return code -> the same code on every rank: ECG_OK if
// all ranks are ok, else the code of the lowest failing rank (the local
// message is kept on that rank, the others name it).  `agree` words (e.g.
// field, size) must match across ranks, else ECG_ERR_INVALID everywhere.
int comm_agree(ecg_ctx* ctx, int local_rc, const uint64_t* agree, int n_agree, const char* what, hipStream_t s);
// Bases [x, y] -> a new device buffer in the bucket kernels' layout,
// registered in the process-wide prepared-bases registry (msm.hip).
// How the bucket kernels read d_bases: the boundary [x, y] layout, prepared
// records (ecg_msm_prepare_bases), or a window table (ecg_msm_prepare_table):
// tab_c > 0, record i W + k = 2^(k tab_c) P_i for the tab_n bases, k < W.
struct BaseForm {
  bool prepared = false;
  uint32_t tab_c = 0;
  size_t tab_n = 0;
};

// tab_c > 0: also the window table (rows 2^(k tab_c) P, ecg_msm_prepare_table).
int msm_prepare_run(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n, uint32_t tab_c, void** d_out,
                    hipStream_t s);
// Release a prepared buffer (its header allocation) if p is one: true when
// handled, false for any other pointer (the caller frees it).
bool msm_prepared_free(void* p);
size_t msm_prepared_stride(int curve_id, uint32_t tab_c);  // bytes per base of a prepared buffer
// Plan of a one-task MSM of n terms (window_bits = 0: automatic): window
// bits, windows, and how the sorted entries are grouped (ECG_SORT_* in ecgpu.h).
int msm_plan_info_run(int curve_id, size_t n, uint32_t window_bits, uint32_t* c, uint32_t* windows,
                      int* sort_mode);
// Window size of an automatic window table for n-term MSMs.
uint32_t msm_table_window_auto(int curve_id, size_t n);
int msm_batch_run(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n_bases, const void* d_scalars,
                  int scalar_mont, size_t line_len, size_t n_chunks, uint32_t window_bits, uint64_t* out_jac,
                  hipStream_t s);
int point_sum_host(int curve_id, const uint64_t* points, size_t count, uint64_t* out_jac);
int msm_pass_terms_run(const ecg_ctx* ctx, int curve_id, size_t* out);
// MSM over host slices, uploads pipelined with compute (msm_host_t)
// Cold fill of a base-cache entry inside the pipelined MSM: pass by pass the
// host bases (ark Affine records or [x, y]) go up with the scalars and are
// converted on the device into the prepared buffer `dst` (msm_prepared_alloc,
// n records), which the pass then reads.
struct MsmFill {
  const void* h_bases = nullptr;
  int ark = 0;
  int curve_id = 0;
};
// bases_resident: `bases` is a device prepared buffer (only the scalars travel);
// with fill, that buffer is filled from fill->h_bases on the way.
int msm_host_run(ecg_ctx* ctx, int curve_id, const void* bases, int bases_resident, const void* h_scalars, size_t n,
                 int scalar_mont, uint64_t* out_jac, ecg_abort_cb abort_cb, void* user,
                 const MsmFill* fill = nullptr);
int msm_prepared_alloc(ecg_ctx* ctx, int curve_id, size_t n, uint32_t tab_c, void** d_out, hipStream_t s);
int gen_bases_run(ecg_ctx* ctx, int curve_id, const uint64_t* a, const uint64_t* b, size_t n,
                  void* d_out, hipStream_t s);

// u64 words per point coordinate: Fq (G1) or Fq2 (G2); the largest is BLS12-381 G2.
constexpr int ECG_MAX_COORD_U64 = 12;
inline int fq_limbs64(int curve_id) {
  switch (curve_id) {
    case ECG_CURVE_BLS12_381: return 6;
    case ECG_CURVE_BN254: return 4;
    case ECG_CURVE_BLS12_381_G2: return 12;
    case ECG_CURVE_BN254_G2: return 8;
    default: return 0;
  }
}
inline bool curve_valid(int curve_id) { return fq_limbs64(curve_id) != 0; }

}  // namespace ecg
