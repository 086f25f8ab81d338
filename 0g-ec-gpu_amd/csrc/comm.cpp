// Multi-GPU exchange over RCCL (xGMI), one process per GPU.
//
// The reference's multi-device paths are host threads over devices of one
// process (multiexp.rs:324-367, fft.rs:211-246) with a CPU fold of the
// per-device partial points.  Here each rank owns one MI355X and one ecg_ctx;
// RCCL (linked from /opt/rocm, the same HIP runtime as the rest of the
// library) moves device buffers directly:
//   * MSM: ncclAllGather of the per-rank Jacobian partial (3 x Lq u64),
//     then the EC fold (RCCL has no EC-add reduction);
//   * one NTT split over ranks: three equal-split ncclAllToAll (dfft.hip).
// Rendezvous: the 128-byte ncclUniqueId travels through the caller's
// launcher (ecgpu.dist.HostGroup in bench.py: one authenticated local socket
// per rank, no torch in the process).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "ctx.hpp"

namespace ecg {

#define ECG_NCCL(call)                                                                             \
  do {                                                                                             \
    ncclResult_t r_ = (call);                                                                      \
    if (r_ != ncclSuccess) {                                                                       \
      ::ecg::set_error("RCCL error %s at %s:%d", ncclGetErrorString(r_), __FILE__, __LINE__);      \
      return ECG_ERR_RCCL;                                                                         \
    }                                                                                              \
  } while (0)

int comm_alltoall(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes_per_peer, hipStream_t s) {
  if (ctx->comm_size > 1 && !ctx->comm) {
    set_error("comm_alltoall: %d ranks but no communicator", ctx->comm_size);
    return ECG_ERR_RCCL;
  }
  if (ctx->comm_size == 1) {  // one rank: the exchange is a copy
    ECG_HIP(hipMemcpyAsync(d_recv, d_send, bytes_per_peer * ctx->comm_size, hipMemcpyDeviceToDevice, s));
    return ECG_OK;
  }
  ECG_NCCL(ncclAllToAll(d_send, d_recv, bytes_per_peer, ncclUint8, (ncclComm_t)ctx->comm, s));
  return ECG_OK;
}

void comm_free(ecg_ctx* ctx) {
  if (ctx->comm) (void)ncclCommDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  ctx->comm_size = 1;
  ctx->comm_rank = 0;
}

int comm_allgather(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes, hipStream_t s) {
  if (ctx->comm_size > 1 && !ctx->comm) {
    set_error("comm_allgather: %d ranks but no communicator", ctx->comm_size);
    return ECG_ERR_RCCL;
  }
  if (ctx->comm_size == 1) {
    ECG_HIP(hipMemcpyAsync(d_recv, d_send, bytes, hipMemcpyDeviceToDevice, s));
    return ECG_OK;
  }
  ECG_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, (ncclComm_t)ctx->comm, s));
  return ECG_OK;
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
  ECG_NCCL(ncclGetUniqueId(&id));
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return ECG_OK;
}

int ecg_comm_init(ecg_ctx* ctx, int nranks, int rank, const uint8_t* unique_id) {
  ECG_ENTER(ctx);
  if (nranks < 1 || rank < 0 || rank >= nranks || (!unique_id && nranks > 1)) {
    set_error("ecg_comm_init: bad arguments (nranks %d, rank %d)", nranks, rank);
    return ECG_ERR_INVALID;
  }
  comm_free(ctx);  // back to the single-rank state until the new communicator exists
  if (nranks == 1) return ECG_OK;
  ncclUniqueId id;
  memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c;
  ECG_NCCL(ncclCommInitRank(&c, nranks, id, rank));
  ctx->comm = c;
  ctx->comm_size = nranks;
  ctx->comm_rank = rank;
  return ECG_OK;
}

void ecg_comm_destroy(ecg_ctx* ctx) {
  if (!ctx || !ctx->comm) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  comm_free(ctx);
}

int ecg_comm_allgather(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes) {
  ECG_ENTER(ctx);
  ECG_TRY(comm_allgather(ctx, d_send, d_recv, bytes, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return ECG_OK;
}

int ecg_comm_alltoall(ecg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes_per_peer) {
  ECG_ENTER(ctx);
  ECG_TRY(comm_alltoall(ctx, d_send, d_recv, bytes_per_peer, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return ECG_OK;
}

// MSM over this rank's shard; the per-rank partials are all-gathered over
// RCCL and folded, so every rank returns the full result.
int ecg_msm_dist(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n_local,
                 uint64_t* out_jac) {
  ECG_ENTER(ctx);
  if (!out_jac || ((!d_bases || !d_scalars) && n_local)) {
    set_error("ecg_msm_dist: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  hipStream_t s = ctx->stream;
  const size_t pb = 3 * (size_t)fq_limbs64(curve_id) * 8;
  uint64_t part[3 * ECG_MAX_COORD_U64];
  ECG_TRY(msm_run(ctx, curve_id, d_bases, d_scalars, n_local, part, s, nullptr, nullptr));
  void *d_part, *d_all;
  ECG_TRY(ws_get(ctx, "dist_part", pb, &d_part));
  ECG_TRY(ws_get(ctx, "dist_all", pb * ctx->comm_size, &d_all));
  ECG_HIP(hipMemcpyAsync(d_part, part, pb, hipMemcpyHostToDevice, s));
  ECG_TRY(comm_allgather(ctx, d_part, d_all, pb, s));
  std::vector<uint64_t> all(pb / 8 * ctx->comm_size);
  ECG_HIP(hipMemcpyAsync(all.data(), d_all, pb * ctx->comm_size, hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  ECG_TRY(point_sum_host(curve_id, all.data(), ctx->comm_size, out_jac));  // multiexp.rs:394-397
  return kt_collect(ctx);
}

// One NTT of 2^log_n points block-distributed over the communicator's ranks
// (this rank holds points [rank*m, (rank+1)*m), m = 2^log_n / size); in place.
int ecg_fft_dist(ecg_ctx* ctx, int field_id, void* d_local, const uint64_t* omega, uint32_t log_n) {
  ECG_ENTER(ctx);
  if (!d_local || !omega) {
    set_error("ecg_fft_dist: null pointer");
    return ECG_ERR_INVALID;
  }
  ECG_TRY(dfft_run(ctx, field_id, d_local, omega, log_n, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return kt_collect(ctx);
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
