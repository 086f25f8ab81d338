// Multi-GPU exchange over RCCL (xGMI), one process per GPU.
//
// The reference's multi-device paths are host threads over devices of one
// process (multiexp.rs:324-367, fft.rs:211-246) with a CPU fold of the
// per-device partial points.  Here each rank owns one MI355X and one ecg_ctx;
// RCCL (linked from /opt/rocm, the same HIP runtime as the rest of the
// library) moves device buffers directly:
//   * MSM: ncclAllGather of the per-rank [status | Jacobian partial] record,
//     then the EC fold (RCCL has no EC-add reduction);
//   * one NTT split over ranks: three equal-split ncclAllToAll (dfft.hip),
//     with status exchanges before the first and the last.
// Rendezvous: the 128-byte ncclUniqueId travels through the caller's
// launcher (ecgpu.dist.HostGroup in bench.py: one authenticated local socket
// per rank, no torch in the process).
//
// Failure semantics.  The reference stops every device at the first error
// (first-writer-wins result, multiexp.rs:345-365, fft.rs:218-245).  Across
// processes the equivalent is that no rank may leave its peers inside a
// collective: every distributed call exchanges each rank's status before its
// payload collectives (comm_agree, or the status word of the MSM record), so
// a local failure becomes the same error on every rank.  What a status
// exchange cannot cover -- a peer that crashed, or a device fault mid-flight
// -- is bounded by a deadline: the communicator is non-blocking, every call
// and every wait polls ncclCommGetAsyncError against it, and on expiry the
// communicator is aborted (ncclCommAbort) and the call returns an error.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ctx.hpp"
#include "msm_ops.hpp"

namespace ecg {

namespace {

constexpr uint32_t DEFAULT_TIMEOUT_MS = 300000;

uint32_t comm_timeout(const ecg_ctx* ctx) {
  if (ctx->comm_timeout_ms) return ctx->comm_timeout_ms;
  const char* e = getenv("ECG_COMM_TIMEOUT_S");
  const long v = e ? atol(e) : 0;
  return v > 0 && v < 4000000 ? (uint32_t)(v * 1000) : DEFAULT_TIMEOUT_MS;
}

using Clock = std::chrono::steady_clock;

struct Deadline {
  Clock::time_point end;
  int polls = 0;
  explicit Deadline(uint32_t ms) : end(Clock::now() + std::chrono::milliseconds(ms)) {}
  bool expired() const { return Clock::now() >= end; }
  // spin briefly (small collectives finish in tens of us), then back off
  void pause() {
    if (++polls < 200)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(polls < 2000 ? 20 : 200));
  }
};

bool host_transport(const ecg_ctx* ctx) { return ctx->xchg != nullptr; }

// Abort the RCCL communicator after a failure or a timeout: its kernels stop,
// later distributed calls are refused (comm_size > 1, no communicator).
void comm_abort(ecg_ctx* ctx) {
  if (ctx->comm) (void)ncclCommAbort((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
}

int rccl_fail(ecg_ctx* ctx, ncclResult_t r, const char* what) {
  set_error("%s: RCCL error %s (%s); communicator aborted", what, ncclGetErrorString(r),
            ncclGetLastError((ncclComm_t)ctx->comm));
  comm_abort(ctx);
  return ECG_ERR_RCCL;
}

// A call on a non-blocking communicator returns ncclInProgress while it is
// still being set up (connections to peers are made lazily): poll its state
// until it settles, under the deadline.
int rccl_settle(ecg_ctx* ctx, ncclResult_t r, const char* what) {
  Deadline dl(comm_timeout(ctx));
  while (r == ncclInProgress) {
    if (dl.expired()) {
      set_error("%s: RCCL call still in progress after %u ms (a peer rank failed or never arrived); "
                "communicator aborted", what, comm_timeout(ctx));
      comm_abort(ctx);
      return ECG_ERR_RCCL;
    }
    dl.pause();
    if (ncclCommGetAsyncError((ncclComm_t)ctx->comm, &r) != ncclSuccess) r = ncclSystemError;
  }
  return r == ncclSuccess ? ECG_OK : rccl_fail(ctx, r, what);
}

int need_comm(ecg_ctx* ctx, const char* what) {
  if (ctx->comm_size > 1 && !ctx->comm && !ctx->xchg) {
    set_error("%s: %d ranks but no communicator (never initialised, or aborted after a failure)", what,
              ctx->comm_size);
    return ECG_ERR_RCCL;
  }
  return ECG_OK;
}

// Host transport: stage through host memory, the caller's callback moves it.
int host_exchange(ecg_ctx* ctx, int op, const void* d_send, void* d_recv, size_t bytes, hipStream_t s,
                  const char* what) {
  const size_t P = (size_t)ctx->comm_size;
  std::vector<uint8_t> send(op == ECG_XCHG_ALLGATHER ? bytes : bytes * P), recv(bytes * P);
  if (!send.empty()) ECG_HIP(hipMemcpyAsync(send.data(), d_send, send.size(), hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  if (ctx->xchg(op, send.data(), recv.data(), bytes, ctx->xchg_user) != 0) {
    set_error("%s: the host transport failed", what);
    return ECG_ERR_RCCL;
  }
  if (!recv.empty()) ECG_HIP(hipMemcpyAsync(d_recv, recv.data(), recv.size(), hipMemcpyHostToDevice, s));
  ECG_HIP(hipStreamSynchronize(s));
  return ECG_OK;
}

}  // namespace

#define ECG_NCCL(ctx, call, what)                                    \
  do {                                                               \
    ncclResult_t r_ = (call);                                        \
    if (r_ != ncclSuccess) ECG_TRY(rccl_settle((ctx), r_, (what)));  \
  } while (0)

int comm_wait(ecg_ctx* ctx, hipStream_t s, const char* what) {
  if (!ctx->comm) {  // no RCCL work can be pending: a plain wait
    ECG_HIP(hipStreamSynchronize(s));
    return ECG_OK;
  }
  Deadline dl(comm_timeout(ctx));
  for (;;) {
    hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return ECG_OK;
    if (e != hipErrorNotReady) {
      set_error("%s: HIP error %s while waiting for the exchange; communicator aborted", what, hipGetErrorName(e));
      comm_abort(ctx);
      return ECG_ERR_HIP;
    }
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError((ncclComm_t)ctx->comm, &ae) != ncclSuccess) ae = ncclSystemError;
    if (ae != ncclSuccess && ae != ncclInProgress) return rccl_fail(ctx, ae, what);
    if (dl.expired()) {
      set_error("%s: no progress within %u ms (a peer rank failed or never arrived); communicator aborted", what,
                comm_timeout(ctx));
      comm_abort(ctx);
      return ECG_ERR_RCCL;
    }
    dl.pause();
  }
}

int comm_alltoall(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes_per_peer, hipStream_t s) {
  ECG_TRY(need_comm(ctx, "alltoall"));
  if (host_transport(ctx)) return host_exchange(ctx, ECG_XCHG_ALLTOALL, d_send, d_recv, bytes_per_peer, s, "alltoall");
  if (!ctx->comm) {  // one rank: the exchange is a copy
    ECG_HIP(hipMemcpyAsync(d_recv, d_send, bytes_per_peer * ctx->comm_size, hipMemcpyDeviceToDevice, s));
    return ECG_OK;
  }
  ECG_NCCL(ctx, ncclAllToAll(d_send, d_recv, bytes_per_peer, ncclUint8, (ncclComm_t)ctx->comm, s), "alltoall");
  return ECG_OK;
}

int comm_allgather(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes, hipStream_t s) {
  ECG_TRY(need_comm(ctx, "allgather"));
  if (host_transport(ctx)) return host_exchange(ctx, ECG_XCHG_ALLGATHER, d_send, d_recv, bytes, s, "allgather");
  if (!ctx->comm) {
    ECG_HIP(hipMemcpyAsync(d_recv, d_send, bytes, hipMemcpyDeviceToDevice, s));
    return ECG_OK;
  }
  ECG_NCCL(ctx, ncclAllGather(d_send, d_recv, bytes, ncclUint8, (ncclComm_t)ctx->comm, s), "allgather");
  return ECG_OK;
}

void comm_free(ecg_ctx* ctx) {
  if (ctx->comm) (void)ncclCommDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  if (ctx->comm_rec) (void)hipFree(ctx->comm_rec);
  ctx->comm_rec = nullptr;
  ctx->comm_rec_bytes = 0;
  ctx->xchg = nullptr;
  ctx->xchg_user = nullptr;
  ctx->comm_size = 1;
  ctx->comm_rank = 0;
}

// Status words ride in fixed-size records so ranks that disagree on the
// call's arguments still exchange equal byte counts.
constexpr int AGREE_WORDS = 4;
// The largest status record: the MSM's [rc | curve | Jacobian partial].
constexpr size_t REC_MAX_BYTES = (2 + 3 * (size_t)ECG_MAX_COORD_U64) * 8;

// All-gather of one small host record per rank, for the status exchanges.
// Nothing here allocates device memory: the host transport moves the host
// records itself, and RCCL stages them through ctx->comm_rec, reserved at
// ecg_comm_init.  So a rank whose call failed on a workspace allocation (or
// anything else local) still joins the exchange and its peers learn of the
// failure at once instead of waiting out the deadline.
int comm_exchange_rec(ecg_ctx* ctx, const void* h_send, void* h_recv, size_t bytes, hipStream_t s,
                      const char* what) {
  ECG_TRY(need_comm(ctx, what));
  const size_t P = (size_t)ctx->comm_size;
  if (host_transport(ctx)) {
    if (ctx->xchg(ECG_XCHG_ALLGATHER, h_send, h_recv, bytes, ctx->xchg_user) != 0) {
      set_error("%s: the host transport failed", what);
      return ECG_ERR_RCCL;
    }
    return ECG_OK;
  }
  if (!ctx->comm) {  // one rank, no communicator
    memcpy(h_recv, h_send, bytes);
    return ECG_OK;
  }
  if (bytes > REC_MAX_BYTES || !ctx->comm_rec || ctx->comm_rec_bytes < REC_MAX_BYTES + bytes * P) {
    set_error("%s: status record of %zu bytes does not fit the reserved staging", what, bytes);
    return ECG_ERR_INVALID;
  }
  uint8_t* d_rec = (uint8_t*)ctx->comm_rec;
  uint8_t* d_all = d_rec + REC_MAX_BYTES;
  ECG_HIP(hipMemcpyAsync(d_rec, h_send, bytes, hipMemcpyHostToDevice, s));
  ECG_TRY(comm_allgather(ctx, d_rec, d_all, bytes, s));
  ECG_TRY(comm_wait(ctx, s, what));
  ECG_HIP(hipMemcpyAsync(h_recv, d_all, bytes * P, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  return ECG_OK;
}

int comm_agree(ecg_ctx* ctx, int local_rc, const uint64_t* agree, int n_agree, const char* what, hipStream_t s) {
  const int P = ctx->comm_size;
  if (P == 1 && !ctx->comm) return local_rc;
  ECG_TRY(need_comm(ctx, what));
  const std::string local_msg = local_rc != ECG_OK ? last_error_text() : "";
  uint64_t rec[1 + AGREE_WORDS] = {(uint64_t)(int64_t)local_rc, 0, 0, 0, 0};
  for (int i = 0; i < n_agree && i < AGREE_WORDS; i++) rec[1 + i] = agree[i];
  if (local_rc != ECG_OK) (void)hipStreamSynchronize(s);  // the failed step's work is done or abandoned
  std::vector<uint64_t> all((1 + AGREE_WORDS) * (size_t)P);
  ECG_TRY(comm_exchange_rec(ctx, rec, all.data(), sizeof rec, s, what));
  for (int r = 0; r < P; r++) {
    const int rc = (int)(int64_t)all[(size_t)r * (1 + AGREE_WORDS)];
    if (rc == ECG_OK) continue;
    if (r == ctx->comm_rank)
      set_error("%s", local_msg.c_str());
    else
      set_error("%s: rank %d of %d failed (rc=%d); every rank stops", what, r, P, rc);
    return rc;
  }
  for (int r = 0; r < P; r++)
    if (memcmp(&all[(size_t)r * (1 + AGREE_WORDS) + 1], &rec[1], AGREE_WORDS * 8) != 0) {
      set_error("%s: rank %d was called with other arguments than rank %d (field / curve / size differ)", what, r,
                ctx->comm_rank);
      return ECG_ERR_INVALID;
    }
  return ECG_OK;
}

// The per-rank [status | curve | partial] records are all-gathered and, when
// every rank succeeded, the partials folded, so every rank returns the full
// result -- or the same error (the lowest failing rank's).  `rc` and the
// partial in rec come from this rank's local step; nothing here allocates
// (comm_exchange_rec), so a failed local step still joins the exchange.
// `shape` (the grid split's n; 0 for the range split, whose shards may differ)
// rides in the record's curve word, so ranks called with different whole-MSM
// sizes -- whose grid shares would overlap or leave gaps -- all fail.
static int dist_fold_partials(ecg_ctx* ctx, int rc, int curve_id, uint64_t* rec, size_t rec_words, uint64_t* out_jac,
                              hipStream_t s, const char* what, uint64_t shape = 0) {
  const std::string local_msg = rc != ECG_OK ? last_error_text() : "";
  if (rc != ECG_OK) (void)hipStreamSynchronize(s);  // the failed run's work is done or abandoned
  rec[0] = (uint64_t)(int64_t)rc;
  rec[1] = (uint64_t)(uint8_t)curve_id | shape << 8;
  const int P = ctx->comm_size;
  // one exchange, no allocation on this path: every rank joins it whatever
  // its local step did (comm_exchange_rec)
  std::vector<uint64_t> all(rec_words * (size_t)P);
  const auto t_x = std::chrono::steady_clock::now();
  ECG_TRY(comm_exchange_rec(ctx, rec, all.data(), rec_words * 8, s, what));
  ctx->comm_last_xchg_us =
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_x).count();
  for (int r = 0; r < P; r++) {  // the lowest failing rank's code, on every rank
    const int rrc = (int)(int64_t)all[(size_t)r * rec_words];
    if (rrc == ECG_OK) continue;
    if (r == ctx->comm_rank)
      set_error("%s", local_msg.c_str());
    else
      set_error("%s: rank %d of %d failed (rc=%d); every rank stops", what, r, P, rrc);
    return rrc;
  }
  const size_t pw = 3 * (size_t)fq_limbs64(curve_id);
  std::vector<uint64_t> parts(pw * P);
  for (int r = 0; r < P; r++) {
    const uint64_t w = all[(size_t)r * rec_words + 1];
    if (w != rec[1]) {
      set_error("%s: rank %d ran curve %d over n = %llu, this rank curve %d over n = %llu", what, r, (int)(w & 0xff),
                (unsigned long long)(w >> 8), curve_id, (unsigned long long)shape);
      return ECG_ERR_INVALID;
    }
    memcpy(&parts[pw * r], &all[(size_t)r * rec_words + 2], pw * 8);
  }
  ECG_TRY(point_sum_host(curve_id, parts.data(), (size_t)P, out_jac));  // multiexp.rs:394-397
  return kt_collect(ctx);
}

}  // namespace ecg

using namespace ecg;

extern "C" {

int ecg_comm_unique_id(uint8_t* out) {
  if (!out) {
    set_error("ecg_comm_unique_id: null pointer");
    return ECG_ERR_INVALID;
  }
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    set_error("ncclGetUniqueId: %s", ncclGetErrorString(r));
    return ECG_ERR_RCCL;
  }
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return ECG_OK;
}

int ecg_comm_set_timeout(ecg_ctx* ctx, uint32_t ms) {
  ECG_ENTER(ctx);
  ctx->comm_timeout_ms = ms;
  return ECG_OK;
}

int ecg_comm_init(ecg_ctx* ctx, int nranks, int rank, const uint8_t* unique_id) {
  ECG_ENTER(ctx);
  if (nranks < 1 || rank < 0 || rank >= nranks || (!unique_id && nranks > 1)) {
    set_error("ecg_comm_init: bad arguments (nranks %d, rank %d)", nranks, rank);
    return ECG_ERR_INVALID;
  }
  (void)hipStreamSynchronize(ctx->stream);
  comm_free(ctx);  // back to the single-rank state until the new communicator exists
  if (!unique_id) return ECG_OK;  // one rank, no communicator
  // the status-record staging (comm_exchange_rec), before any collective:
  // a rank that cannot allocate it never enters the communicator's init
  {
    const size_t bytes = REC_MAX_BYTES * ((size_t)nranks + 1);
    hipError_t e = hipMalloc(&ctx->comm_rec, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      ctx->comm_rec = nullptr;
      set_error("ecg_comm_init: staging of %zu bytes for the status records failed: %s", bytes, hipGetErrorString(e));
      return ECG_ERR_NOMEM;
    }
    ctx->comm_rec_bytes = bytes;
  }
  ncclUniqueId id;
  memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;  // every wait below runs under the deadline
  ncclComm_t c = nullptr;
  ncclResult_t r = ncclCommInitRankConfig(&c, nranks, id, rank, &cfg);
  // from here on the context is an nranks-rank context: if the communicator
  // fails to come up, comm stays null and need_comm refuses every
  // distributed call until ecg_comm_init runs again (not a silent 1-rank run)
  ctx->comm_size = nranks;
  ctx->comm_rank = rank;
  if (r != ncclSuccess && r != ncclInProgress) {
    set_error("ncclCommInitRankConfig: %s", ncclGetErrorString(r));
    if (c) (void)ncclCommAbort(c);
    return ECG_ERR_RCCL;
  }
  ctx->comm = c;
  return rccl_settle(ctx, r, "ecg_comm_init");
}

int ecg_comm_init_host(ecg_ctx* ctx, int nranks, int rank, ecg_xchg_cb xchg, void* user) {
  ECG_ENTER(ctx);
  if (nranks < 1 || rank < 0 || rank >= nranks || !xchg) {
    set_error("ecg_comm_init_host: bad arguments (nranks %d, rank %d, callback %p)", nranks, rank, (void*)xchg);
    return ECG_ERR_INVALID;
  }
  (void)hipStreamSynchronize(ctx->stream);
  comm_free(ctx);
  ctx->xchg = xchg;
  ctx->xchg_user = user;
  ctx->comm_size = nranks;
  ctx->comm_rank = rank;
  return ECG_OK;
}

int ecg_comm_info(ecg_ctx* ctx, int* nranks, int* rank, int* device, char* bus_id, size_t bus_cap, int* transport) {
  ECG_ENTER(ctx);
  int n = ctx->comm_size, r = ctx->comm_rank, d = ctx->device;
  int t = host_transport(ctx) ? ECG_COMM_HOST : ctx->comm ? ECG_COMM_RCCL : ctx->comm_size > 1 ? ECG_COMM_FAILED
                                                                                                 : ECG_COMM_NONE;
  if (t == ECG_COMM_RCCL) {  // what the communicator itself reports
    ncclComm_t c = (ncclComm_t)ctx->comm;
    if (ncclCommCount(c, &n) != ncclSuccess || ncclCommUserRank(c, &r) != ncclSuccess ||
        ncclCommCuDevice(c, &d) != ncclSuccess) {
      set_error("ecg_comm_info: the RCCL communicator did not answer its queries");
      return ECG_ERR_RCCL;
    }
  }
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (device) *device = d;
  if (transport) *transport = t;
  if (bus_id && bus_cap) {
    bus_id[0] = 0;
    ECG_HIP(hipDeviceGetPCIBusId(bus_id, (int)bus_cap, d));
  }
  return ECG_OK;
}

int ecg_comm_last_exchange(ecg_ctx* ctx, double* us) {
  ECG_ENTER(ctx);
  if (!us) {
    set_error("ecg_comm_last_exchange: null pointer");
    return ECG_ERR_INVALID;
  }
  *us = ctx->comm_last_xchg_us;
  return ECG_OK;
}

void ecg_comm_destroy(ecg_ctx* ctx) {
  if (!ctx) return;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  comm_free(ctx);
}

int ecg_comm_allgather(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes) {
  ECG_ENTER(ctx);
  ECG_TRY(comm_allgather(ctx, d_send, d_recv, bytes, ctx->stream));
  return comm_wait(ctx, ctx->stream, "ecg_comm_allgather");
}

int ecg_comm_alltoall(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes_per_peer) {
  ECG_ENTER(ctx);
  ECG_TRY(comm_alltoall(ctx, d_send, d_recv, bytes_per_peer, ctx->stream));
  return comm_wait(ctx, ctx->stream, "ecg_comm_alltoall");
}


// MSM over this rank's shard (range split), then dist_fold_partials.
int ecg_msm_dist_ex(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n_local,
                    uint64_t* out_jac, ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  hipStream_t s = ctx->stream;
  constexpr size_t PW = 3 * (size_t)ECG_MAX_COORD_U64;  // partial words, the largest curve's
  uint64_t rec[2 + PW] = {};
  static_assert(sizeof rec <= REC_MAX_BYTES, "MSM status record exceeds the reserved staging");
  int rc = ECG_OK;
  if (!out_jac || ((!d_bases || !d_scalars) && n_local)) {
    set_error("ecg_msm_dist: null pointer");
    rc = ECG_ERR_INVALID;
  } else if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    rc = ECG_ERR_INVALID;
  } else if (abort_cb && abort_cb(user)) {
    rc = ECG_ABORTED;
  } else {
    rc = msm_run(ctx, curve_id, d_bases, d_scalars, n_local, rec + 2, s, abort_cb, user);
  }
  if (ctx->comm_size == 1 && !ctx->comm) {  // one rank: the partial is the result
    if (rc != ECG_OK) return rc;
    memcpy(out_jac, rec + 2, 3 * (size_t)fq_limbs64(curve_id) * 8);
    return kt_collect(ctx);
  }
  return dist_fold_partials(ctx, rc, curve_id, rec, 2 + PW, out_jac, s, "ecg_msm_dist");
}

// Grid split: every rank holds all n bases and scalars; rank r runs the r-th
// of comm_size equal ranges of the (window x term) grid of the n-term plan
// (msm_grid_run), then dist_fold_partials.
int ecg_msm_dist_grid_ex(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n,
                         uint64_t* out_jac, ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  hipStream_t s = ctx->stream;
  constexpr size_t PW = 3 * (size_t)ECG_MAX_COORD_U64;
  uint64_t rec[2 + PW] = {};
  int rc = ECG_OK;
  if (!out_jac || ((!d_bases || !d_scalars) && n)) {
    set_error("ecg_msm_dist_grid: null pointer");
    rc = ECG_ERR_INVALID;
  } else if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    rc = ECG_ERR_INVALID;
  } else if (abort_cb && abort_cb(user)) {
    rc = ECG_ABORTED;
  } else {
    kt_reset(ctx, "msm_accumulate");
    rc = msm_grid_run(ctx, curve_id, d_bases, d_scalars, n, ctx->comm_rank, ctx->comm_size, rec + 2, s, abort_cb,
                      user, nullptr);
  }
  if (ctx->comm_size == 1 && !ctx->comm) {
    if (rc != ECG_OK) return rc;
    memcpy(out_jac, rec + 2, 3 * (size_t)fq_limbs64(curve_id) * 8);
    return kt_collect(ctx);
  }
  return dist_fold_partials(ctx, rc, curve_id, rec, 2 + PW, out_jac, s, "ecg_msm_dist_grid", (uint64_t)n);
}

int ecg_msm_dist_grid(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n,
                      uint64_t* out_jac) {
  return ecg_msm_dist_grid_ex(ctx, curve_id, d_bases, d_scalars, n, out_jac, nullptr, nullptr);
}

// One grid piece set of rank `rank` of `nranks` on this context (no
// exchange): the per-rank step of ecg_msm_dist_grid, for callers (and tests
// with several contexts on one device) that fold the partials themselves.
int ecg_msm_grid_part(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n, int rank,
                      int nranks, uint64_t* out_jac, int* pieces) {
  ECG_ENTER(ctx);
  if (!out_jac || ((!d_bases || !d_scalars) && n)) {
    set_error("ecg_msm_grid_part: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  kt_reset(ctx, "msm_accumulate");
  ECG_TRY(msm_grid_run(ctx, curve_id, d_bases, d_scalars, n, rank, nranks, out_jac, ctx->stream, nullptr, nullptr,
                       pieces));
  return kt_collect(ctx);
}

int ecg_msm_dist(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n_local,
                 uint64_t* out_jac) {
  return ecg_msm_dist_ex(ctx, curve_id, d_bases, d_scalars, n_local, out_jac, nullptr, nullptr);
}

// One NTT of 2^log_n points block-distributed over the communicator's ranks
// (this rank holds points [rank*m, (rank+1)*m), m = 2^log_n / size); in place.
int ecg_fft_dist_ex(ecg_ctx* ctx, int field_id, void* d_local, const uint64_t* omega, uint32_t log_n,
                    ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  ECG_TRY(dfft_run(ctx, field_id, d_local, omega, log_n, ctx->stream, abort_cb, user));
  ECG_TRY(comm_wait(ctx, ctx->stream, "ecg_fft_dist"));
  return kt_collect(ctx);
}

int ecg_fft_dist(ecg_ctx* ctx, int field_id, void* d_local, const uint64_t* omega, uint32_t log_n) {
  return ecg_fft_dist_ex(ctx, field_id, d_local, omega, log_n, nullptr, nullptr);
}

// The two local steps of ecg_fft_dist, exposed so a caller (or a test with
// several contexts on one device) can drive the exchanges itself.
int ecg_fft_dist_stage1(ecg_ctx* ctx, int field_id, const void* d_in, void* d_out, const uint64_t* omega,
                        uint32_t nranks, uint32_t rank, uint32_t log_n) {
  ECG_ENTER(ctx);
  if (!d_in || !d_out || !omega) {
    set_error("ecg_fft_dist_stage1: null pointer");
    return ECG_ERR_INVALID;
  }
  ECG_TRY(dfft_stage1(field_id, d_in, d_out, omega, nranks, rank, log_n, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return ECG_OK;
}

int ecg_fft_dist_stage3(ecg_ctx* ctx, const void* d_in, void* d_out, uint32_t nranks, uint32_t log_n) {
  ECG_ENTER(ctx);
  if (!d_in || !d_out) {
    set_error("ecg_fft_dist_stage3: null pointer");
    return ECG_ERR_INVALID;
  }
  ECG_TRY(dfft_stage3(d_in, d_out, nranks, log_n, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return ECG_OK;
}

}  // extern "C"
