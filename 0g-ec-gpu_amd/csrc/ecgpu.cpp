// C ABI of libecgpu.so (include/ecgpu.h): contexts, workspace, errors, the
// host<->device boundary of the reference API, and multi-device dispatch.
//
// Reference mapping (ec-gpu-proxy):
//   ecg_fft        <- SingleFftKernel::radix_fft        (src/fft.rs:50-135)
//   ecg_fft_many   <- FftKernel::radix_fft_many         (src/fft.rs:211-246)
//   ecg_msm        <- SingleMultiexpKernel::multiexp    (src/multiexp.rs:135-236)
//   ecg_msm_multi  <- MultiexpKernel::parallel_multiexp (src/multiexp.rs:324-367)
//                     + multiexp's device fold          (src/multiexp.rs:394-397)
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ctx.hpp"

namespace ecg {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

const char* last_error_text() { return g_err.c_str(); }

int ctx_enter(ecg_ctx* ctx) {
  if (!ctx) {
    set_error("null context");
    return ECG_ERR_INVALID;
  }
  ECG_HIP(hipSetDevice(ctx->device));
  return ECG_OK;
}

int ws_get(ecg_ctx* ctx, const char* name, size_t bytes, void** out) {
  auto& b = ctx->ws[name];
  if (bytes == 0) bytes = 16;
  if (b.bytes < bytes && ctx->mem_limit) {  // ecg_ctx_set_mem_limit
    size_t total = bytes;
    for (const auto& kv : ctx->ws)
      if (&kv.second != &b) total += kv.second.bytes;
    if (total > ctx->mem_limit) {
      set_error("device allocation of %zu bytes for '%s' refused: the context's workspace would reach %zu bytes, "
                "over its limit of %zu (ecg_ctx_set_mem_limit)", bytes, name, total, ctx->mem_limit);
      return ECG_ERR_NOMEM;
    }
  }
  if (b.bytes < bytes) {
    if (b.ptr) {
      // the buffer may still be in use by queued work on any stream the caller
      // chose (pick_stream), not only ctx->stream: drain the device (growth is rare)
      ECG_HIP(hipDeviceSynchronize());
      ECG_HIP(hipFree(b.ptr));
      b.ptr = nullptr;
      b.bytes = 0;
    }
    hipError_t e = hipMalloc(&b.ptr, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("device allocation of %zu bytes for '%s' failed: %s", bytes, name, hipGetErrorString(e));
      b.ptr = nullptr;
      return ECG_ERR_NOMEM;
    }
    b.bytes = bytes;
  }
  *out = b.ptr;
  return ECG_OK;
}

int hws_get(ecg_ctx* ctx, const char* name, size_t bytes, void** out, void** dev) {
  auto& b = ctx->hws[name];
  if (bytes == 0) bytes = 16;
  if (b.bytes < bytes) {
    if (b.ptr) {
      // a queued copy or kernel (on ctx->stream, the caller's stream or the
      // pipeline's copy stream) may still target it: drain the device
      ECG_HIP(hipDeviceSynchronize());
      ECG_HIP(hipHostFree(b.ptr));
      b.ptr = nullptr;
      b.bytes = 0;
    }
    hipError_t e = hipHostMalloc(&b.ptr, bytes, hipHostMallocMapped);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("pinned host allocation of %zu bytes for '%s' failed: %s", bytes, name, hipGetErrorString(e));
      b.ptr = nullptr;
      return ECG_ERR_NOMEM;
    }
    b.bytes = bytes;
  }
  *out = b.ptr;
  if (dev) ECG_HIP(hipHostGetDevicePointer(dev, b.ptr, 0));
  return ECG_OK;
}

void ws_release(ecg_ctx* ctx, const char* name) {
  auto it = ctx->ws.find(name);
  if (it == ctx->ws.end()) return;
  if (it->second.ptr) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(it->second.ptr);
  }
  ctx->ws.erase(it);
}

hipEvent_t ev_take(ecg_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void kt_reset(ecg_ctx* ctx, const char* name) {
  auto& kt = ctx->ktimes[name];
  for (auto& pr : kt.pending) {
    ctx->event_pool.push_back(pr.first);
    ctx->event_pool.push_back(pr.second);
  }
  kt.pending.clear();
  kt.ms = 0.0;
  kt.launches = 0;
}

int kt_begin(ecg_ctx* ctx, const char* name, hipStream_t s) {
  hipEvent_t a = ev_take(ctx), b = ev_take(ctx);
  if (!a || !b) {
    set_error("hipEventCreate failed");
    return ECG_ERR_HIP;
  }
  ECG_HIP(hipEventRecord(a, s));
  ctx->ktimes[name].pending.push_back({a, b});
  return ECG_OK;
}

int kt_end(ecg_ctx* ctx, const char* name, hipStream_t s) {
  auto& kt = ctx->ktimes[name];
  ECG_HIP(hipEventRecord(kt.pending.back().second, s));
  return ECG_OK;
}

int kt_collect(ecg_ctx* ctx) {
  for (auto& kv : ctx->ktimes) {
    auto& kt = kv.second;
    for (auto& pr : kt.pending) {
      ECG_HIP(hipEventSynchronize(pr.second));
      float ms = 0.f;
      ECG_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
      kt.ms += ms;
      kt.launches += 1;
      ctx->event_pool.push_back(pr.first);
      ctx->event_pool.push_back(pr.second);
    }
    kt.pending.clear();
  }
  return ECG_OK;
}

static size_t fr_bytes(int field_id) {
  return (field_id == ECG_FIELD_BLS12_381_FQ) ? 48 : 32;
}

}  // namespace ecg

using namespace ecg;

extern "C" {

const char* ecg_last_error(void) { return g_err.c_str(); }

const char* ecg_version(void) { return "ecgpu-mi355x 0.1.0 (gfx950)"; }

int ecg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int ecg_ctx_create(int device, ecg_ctx** out) {
  if (!out) {
    set_error("ecg_ctx_create: null out pointer");
    return ECG_ERR_INVALID;
  }
  *out = nullptr;
  int n = ecg_device_count();
  if (n <= 0) {
    set_error("No working GPUs found!");  // fft.rs:183, multiexp.rs:305
    return ECG_ERR_NODEV;
  }
  if (device < 0 || device >= n) {
    set_error("ecg_ctx_create: device %d out of range [0, %d)", device, n);
    return ECG_ERR_INVALID;
  }
  ECG_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  ECG_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("ecg_ctx_create: device %d is %s; this build targets gfx950 (MI355X) only", device,
              prop.gcnArchName);
    return ECG_ERR_NODEV;
  }
  ecg_ctx* ctx = new ecg_ctx();
  ctx->device = device;
  ctx->mem_bytes = prop.totalGlobalMem;
  ctx->compute_units = prop.multiProcessorCount;
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    set_error("hipStreamCreate failed: %s", hipGetErrorString(e));
    delete ctx;
    return ECG_ERR_HIP;
  }
  *out = ctx;
  return ECG_OK;
}

static void base_cache_free(ecg_ctx* ctx);

void ecg_ctx_destroy(ecg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->ws)
    if (kv.second.ptr) (void)hipFree(kv.second.ptr);
  for (auto& kv : ctx->hws)
    if (kv.second.ptr) (void)hipHostFree(kv.second.ptr);
  for (auto& kv : ctx->ktimes)
    for (auto& pr : kv.second.pending) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
  base_cache_free(ctx);
  comm_free(ctx);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int ecg_ctx_synchronize(ecg_ctx* ctx) {
  ECG_ENTER(ctx);
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  ECG_HIP(hipDeviceSynchronize());
  return ECG_OK;
}

int ecg_ctx_info(ecg_ctx* ctx, size_t* mem_bytes, int* compute_units) {
  if (!ctx) {
    set_error("null context");
    return ECG_ERR_INVALID;
  }
  if (mem_bytes) *mem_bytes = ctx_mem(ctx);
  if (compute_units) *compute_units = ctx->compute_units;
  return ECG_OK;
}

// ---------------------------------------------------------------- FFT
int ecg_fft_dev(ecg_ctx* ctx, int field_id, void* d_inout, const uint64_t* omega, uint32_t log_n, void* stream) {
  ECG_ENTER(ctx);
  if (!d_inout || !omega) {
    set_error("ecg_fft_dev: null pointer");
    return ECG_ERR_INVALID;
  }
  hipStream_t s = pick_stream(ctx, stream);
  ECG_TRY(ntt_run(ctx, field_id, d_inout, omega, log_n, s, nullptr, nullptr));
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

int ecg_fft(ecg_ctx* ctx, int field_id, uint64_t* inout, const uint64_t* omega, uint32_t log_n,
            ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  if (!inout || !omega) {
    set_error("ecg_fft: null pointer");
    return ECG_ERR_INVALID;
  }
  ECG_TRY(ntt_validate(field_id, log_n));  // before any allocation or copy
  const size_t bytes = ((size_t)1 << log_n) * fr_bytes(field_id);
  void* d;
  ECG_TRY(ws_get(ctx, "fft_io", bytes, &d));
  hipStream_t s = ctx->stream;
  ECG_HIP(hipMemcpyAsync(d, inout, bytes, hipMemcpyHostToDevice, s));  // fft.rs:89
  int rc = ntt_run(ctx, field_id, d, omega, log_n, s, abort_cb, user);
  if (rc != ECG_OK) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  ECG_HIP(hipMemcpyAsync(inout, d, bytes, hipMemcpyDeviceToHost, s));  // fft.rs:129
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

// Same-size transforms with the same omega, back to back in one device buffer
// and run as ONE batched transform (each pass launches every transform's
// tiles together): a 2^16 transform alone is 64 workgroups on 256 CUs.
// Results are identical to one ecg_fft per input.
constexpr size_t FFT_BATCH_BYTES = (size_t)1 << 30;
static int fft_batch(ecg_ctx* ctx, int field_id, uint64_t** inouts, const uint64_t* omega, uint32_t log_n,
                     size_t cnt, ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  ECG_TRY(ntt_validate(field_id, log_n));
  const size_t bytes = ((size_t)1 << log_n) * fr_bytes(field_id);
  void* d;
  ECG_TRY(ws_get(ctx, "fft_io", cnt * bytes, &d));
  hipStream_t s = ctx->stream;
  for (size_t b = 0; b < cnt; b++) {
    ECG_HIP(hipMemcpyAsync((uint8_t*)d + b * bytes, inouts[b], bytes, hipMemcpyHostToDevice, s));  // fft.rs:89
  }
  int rc = ntt_run(ctx, field_id, d, omega, log_n, s, abort_cb, user, (uint32_t)cnt);
  if (rc != ECG_OK) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  for (size_t b = 0; b < cnt; b++)
    ECG_HIP(hipMemcpyAsync(inouts[b], (uint8_t*)d + b * bytes, bytes, hipMemcpyDeviceToHost, s));  // fft.rs:129
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

// Every pointer a *_many call dereferences, checked before any worker starts
// (the batch helpers then only see valid inputs).
static int many_args_ok(const char* what, uint64_t** inouts, const uint64_t* omegas, const uint32_t* log_ns,
                        size_t count) {
  if (!inouts || !omegas || !log_ns) {
    set_error("%s: null pointer", what);
    return ECG_ERR_INVALID;
  }
  for (size_t i = 0; i < count; i++)
    if (!inouts[i]) {
      set_error("%s: null pointer (input %zu)", what, i);
      return ECG_ERR_INVALID;
    }
  return ECG_OK;
}

int ecg_fft_many(ecg_ctx** ctxs, int nctx, int field_id, uint64_t** inouts, const uint64_t* omegas,
                 const uint32_t* log_ns, size_t count, ecg_abort_cb abort_cb, void* user) {
  if (!ctxs || nctx <= 0) {
    set_error("No working GPUs found!");
    return ECG_ERR_NODEV;
  }
  if (count == 0) return ECG_OK;
  ECG_TRY(many_args_ok("ecg_fft_many", inouts, omegas, log_ns, count));
  const size_t chunk = (count + nctx - 1) / nctx;  // fft.rs:216
  std::atomic<int> first_err{ECG_OK};
  std::mutex mu;
  std::string err_msg;
  std::vector<std::thread> th;
  for (int d = 0; d < nctx && (size_t)d * chunk < count; d++) {
    th.emplace_back([&, d]() {
      const size_t i0 = d * chunk, i1 = std::min(count, i0 + chunk);
      for (size_t i = i0, j; i < i1; i = j) {
        if (first_err.load() != ECG_OK) break;  // fft.rs:233-235
        // the run of inputs sharing this one's size and omega (fft_batch)
        const size_t one = ((size_t)1 << std::min(log_ns[i], 40u)) * fr_bytes(field_id);
        j = i + 1;
        while (j < i1 && log_ns[j] == log_ns[i] && memcmp(omegas + 4 * j, omegas + 4 * i, 32) == 0 &&
               (j - i + 1) * one <= FFT_BATCH_BYTES)
          j++;
        int rc = j - i == 1 ? ecg_fft(ctxs[d], field_id, inouts[i], omegas + 4 * i, log_ns[i], abort_cb, user)
                            : fft_batch(ctxs[d], field_id, inouts + i, omegas + 4 * i, log_ns[i], j - i, abort_cb, user);
        if (rc != ECG_OK) {
          int expected = ECG_OK;
          if (first_err.compare_exchange_strong(expected, rc)) {
            std::lock_guard<std::mutex> g(mu);
            err_msg = g_err;
          }
          break;
        }
      }
    });
  }
  for (auto& t : th) t.join();
  if (first_err.load() != ECG_OK) g_err = err_msg;
  return first_err.load();
}

// ---------------------------------------------------------------- EC-FFT
int ecg_ec_fft(ecg_ctx* ctx, int curve_id, uint64_t* inout_jac, const uint64_t* omega, uint32_t log_n,
               ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  if (!inout_jac || !omega) {
    set_error("ecg_ec_fft: null pointer");
    return ECG_ERR_INVALID;
  }
  ECG_TRY(ecfft_validate(curve_id, log_n));  // before any allocation or copy
  const size_t bytes = ((size_t)1 << log_n) * 3 * fq_limbs64(curve_id) * 8;
  void* d;
  ECG_TRY(ws_get(ctx, "ecfft_io", bytes, &d));
  hipStream_t s = ctx->stream;
  ECG_HIP(hipMemcpyAsync(d, inout_jac, bytes, hipMemcpyHostToDevice, s));  // ec_fft.rs:103
  int rc = ecfft_run(ctx, curve_id, d, omega, log_n, s, abort_cb, user);
  if (rc != ECG_OK) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  ECG_HIP(hipMemcpyAsync(inout_jac, d, bytes, hipMemcpyDeviceToHost, s));  // ec_fft.rs:158
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

int ecg_ec_fft_dev(ecg_ctx* ctx, int curve_id, void* d_inout_jac, const uint64_t* omega, uint32_t log_n,
                   void* stream) {
  ECG_ENTER(ctx);
  if (!d_inout_jac || !omega) {
    set_error("ecg_ec_fft_dev: null pointer");
    return ECG_ERR_INVALID;
  }
  hipStream_t s = pick_stream(ctx, stream);
  ECG_TRY(ecfft_run(ctx, curve_id, d_inout_jac, omega, log_n, s, nullptr, nullptr));
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

// Same-size EC-FFTs with the same omega, back to back and run as ONE batched
// transform (every stage launches the whole run's butterflies): the small
// transforms 0g runs are latency-bound at under one wave per SIMD each.
static size_t ecfft_batch_points() {  // points per batched run (A/B: ECG_ECFFT_BATCH_LOG)
  static const size_t v = [] {
    // clamped to [1, 24]: batch << log_n and the stores' counts stay below 2^32 points
    const char* e = getenv("ECG_ECFFT_BATCH_LOG");
    const int v = e ? atoi(e) : 20;
    return (size_t)1 << (v >= 1 && v <= 24 ? v : 20);
  }();
  return v;
}
static int ec_fft_batch(ecg_ctx* ctx, int curve_id, uint64_t** inouts, const uint64_t* omega, uint32_t log_n,
                        size_t cnt, ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  ECG_TRY(ecfft_validate(curve_id, log_n));
  const size_t bytes = ((size_t)1 << log_n) * 3 * fq_limbs64(curve_id) * 8;
  void* d;
  ECG_TRY(ws_get(ctx, "ecfft_io", cnt * bytes, &d));
  hipStream_t s = ctx->stream;
  for (size_t b = 0; b < cnt; b++) {
    ECG_HIP(hipMemcpyAsync((uint8_t*)d + b * bytes, inouts[b], bytes, hipMemcpyHostToDevice, s));  // ec_fft.rs:103
  }
  int rc = ecfft_run(ctx, curve_id, d, omega, log_n, s, abort_cb, user, (uint32_t)cnt);
  if (rc != ECG_OK) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  for (size_t b = 0; b < cnt; b++)
    ECG_HIP(hipMemcpyAsync(inouts[b], (uint8_t*)d + b * bytes, bytes, hipMemcpyDeviceToHost, s));  // ec_fft.rs:158
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

int ecg_ec_fft_many(ecg_ctx** ctxs, int nctx, int curve_id, uint64_t** inouts, const uint64_t* omegas,
                    const uint32_t* log_ns, size_t count, ecg_abort_cb abort_cb, void* user) {
  if (!ctxs || nctx <= 0) {
    set_error("No working GPUs found!");  // ec_fft.rs:207
    return ECG_ERR_NODEV;
  }
  if (count == 0) return ECG_OK;
  ECG_TRY(many_args_ok("ecg_ec_fft_many", inouts, omegas, log_ns, count));
  const size_t chunk = (count + nctx - 1) / nctx;  // ec_fft.rs:231
  std::atomic<int> first_err{ECG_OK};
  std::mutex mu;
  std::string err_msg;
  std::vector<std::thread> th;
  for (int d = 0; d < nctx && (size_t)d * chunk < count; d++) {
    th.emplace_back([&, d]() {
      const size_t i0 = d * chunk, i1 = std::min(count, i0 + chunk);
      for (size_t i = i0, j; i < i1; i = j) {
        if (first_err.load() != ECG_OK) break;  // ec_fft.rs:249-251
        // the run of inputs sharing this one's size and omega (ec_fft_batch)
        const size_t one = (size_t)1 << std::min(log_ns[i], 40u);
        j = i + 1;
        while (j < i1 && log_ns[j] == log_ns[i] && memcmp(omegas + 4 * j, omegas + 4 * i, 32) == 0 &&
               (j - i + 1) * one <= ecfft_batch_points())
          j++;
        int rc = j - i == 1
                     ? ecg_ec_fft(ctxs[d], curve_id, inouts[i], omegas + 4 * i, log_ns[i], abort_cb, user)
                     : ec_fft_batch(ctxs[d], curve_id, inouts + i, omegas + 4 * i, log_ns[i], j - i, abort_cb, user);
        if (rc != ECG_OK) {
          int expected = ECG_OK;
          if (first_err.compare_exchange_strong(expected, rc)) {
            std::lock_guard<std::mutex> g(mu);
            err_msg = g_err;
          }
          break;
        }
      }
    });
  }
  for (auto& t : th) t.join();
  if (first_err.load() != ECG_OK) g_err = err_msg;
  return first_err.load();
}

// ---------------------------------------------------------------- MSM
static int msm_host(ecg_ctx* ctx, int curve_id, const uint64_t* bases_xy, const uint64_t* scalars, size_t n,
                    uint64_t* out_jac, ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  if ((!bases_xy || !scalars) && n) {
    set_error("ecg_msm: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  // multiexp.rs:163-164 copies the slices in; here the copies are pipelined
  // with the compute pass by pass (msm_host_t)
  ECG_TRY(msm_host_run(ctx, curve_id, bases_xy, 0, scalars, n, 0, out_jac, abort_cb, user));
  return kt_collect(ctx);
}

int ecg_msm(ecg_ctx* ctx, int curve_id, const uint64_t* bases_xy, const uint64_t* scalars, size_t n,
            uint64_t* out_jac, ecg_abort_cb abort_cb, void* user) {
  if (!out_jac) {
    set_error("ecg_msm: null output");
    return ECG_ERR_INVALID;
  }
  return msm_host(ctx, curve_id, bases_xy, scalars, n, out_jac, abort_cb, user);
}

int ecg_msm_dev(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n, void* out_jac,
                int out_on_device, void* stream) {
  ECG_ENTER(ctx);
  if (!out_jac || ((!d_bases || !d_scalars) && n)) {
    set_error("ecg_msm_dev: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  hipStream_t s = pick_stream(ctx, stream);
  uint64_t host_out[3 * ECG_MAX_COORD_U64];
  const size_t ob = 3 * (size_t)fq_limbs64(curve_id) * 8;
  ECG_TRY(msm_run(ctx, curve_id, d_bases, d_scalars, n, host_out, s, nullptr, nullptr));
  if (out_on_device) {
    ECG_HIP(hipMemcpyAsync(out_jac, host_out, ob, hipMemcpyHostToDevice, s));
  } else {
    memcpy(out_jac, host_out, ob);
  }
  ECG_HIP(hipStreamSynchronize(s));
  return kt_collect(ctx);
}

int ecg_msm_prepare_bases(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n, void** d_prepared) {
  ECG_ENTER(ctx);
  if (!d_prepared || (!d_bases && n)) {
    set_error("ecg_msm_prepare_bases: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("prepare_bases: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  if (n > 0x7fffffffull) {
    set_error("prepare_bases: at most 2^31-1 bases");
    return ECG_ERR_INVALID;
  }
  *d_prepared = nullptr;
  return msm_prepare_run(ctx, curve_id, d_bases, n, 0, d_prepared, ctx->stream);
}

size_t ecg_msm_prepared_stride(int curve_id, uint32_t window_bits) {
  return curve_valid(curve_id) ? msm_prepared_stride(curve_id, window_bits) : 0;
}

uint32_t ecg_msm_table_window(int curve_id, size_t n) {
  if (!curve_valid(curve_id)) return 0;
  return msm_table_window_auto(curve_id, n);
}

int ecg_msm_prepare_table(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n, uint32_t window_bits,
                          void** d_prepared) {
  ECG_ENTER(ctx);
  if (!d_prepared || (!d_bases && n)) {
    set_error("ecg_msm_prepare_table: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("prepare_table: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  if (n > 0x7fffffffull) {
    set_error("prepare_table: at most 2^31-1 bases");
    return ECG_ERR_INVALID;
  }
  *d_prepared = nullptr;
  const uint32_t c = window_bits ? window_bits : msm_table_window_auto(curve_id, n);
  return msm_prepare_run(ctx, curve_id, d_bases, n, c ? c : 2, d_prepared, ctx->stream);
}

int ecg_multiple_multiexp(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n_bases, const uint64_t* scalars,
                          int scalars_on_device, int scalars_montgomery, size_t line_len, size_t num_chunks,
                          uint32_t window_bits, uint64_t* out_jac) {
  ECG_ENTER(ctx);
  if (!out_jac || (n_bases && (!d_bases || !scalars))) {
    set_error("ecg_multiple_multiexp: null pointer");
    return ECG_ERR_INVALID;
  }
  hipStream_t s = ctx->stream;
  const void* d_sc = scalars;
  if (!scalars_on_device && n_bases) {  // multiexp.rs:64 in_ref_slice(&exponents)
    void* d;
    ECG_TRY(ws_get(ctx, "mmsm_scalars", line_len * 32, &d));
    ECG_HIP(hipMemcpyAsync(d, scalars, line_len * 32, hipMemcpyHostToDevice, s));
    d_sc = d;
  }
  int rc = msm_batch_run(ctx, curve_id, d_bases, n_bases, d_sc, scalars_montgomery, line_len, num_chunks,
                         window_bits, out_jac, s);
  (void)hipStreamSynchronize(s);
  if (rc != ECG_OK) return rc;
  return kt_collect(ctx);
}

// Cached bases are prepared buffers (registry-owned); release accordingly.
static void base_cache_release(void* dev) {
  if (dev && !msm_prepared_free(dev)) (void)hipFree(dev);
}

static void base_cache_free(ecg_ctx* ctx) {
  for (auto& e : ctx->base_cache) base_cache_release(e.dev);
  ctx->base_cache.clear();
}

void ecg_base_cache_clear(ecg_ctx* ctx) {
  if (!ctx) return;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  base_cache_free(ctx);
}

size_t ecg_base_cache_keys(ecg_ctx* ctx, const void** out, size_t cap) {
  if (!ctx) return 0;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  const size_t n = ctx->base_cache.size();
  for (size_t k = 0; k < n && k < cap && out; k++) out[k] = ctx->base_cache[k].host;
  return n;
}

int ecg_msm_plan_info(int curve_id, size_t n, uint32_t window_bits, uint32_t* c, uint32_t* windows,
                      int* sort_mode) {
  if (!c || !windows || !sort_mode) {
    set_error("ecg_msm_plan_info: null pointer");
    return ECG_ERR_INVALID;
  }
  return msm_plan_info_run(curve_id, n, window_bits, c, windows, sort_mode);
}

// FNV-1a over up to 16 evenly spaced host records (first and last included):
// a cache hit must also match the content the entry was uploaded from, so a
// different array that reuses a freed array's address is not served stale
// bases (the caller must still not mutate a cached array in place).
static uint64_t bases_fingerprint(const void* host, size_t n, size_t rec_bytes) {
  uint64_t h = 1469598103934665603ull ^ n;
  if (!n) return h;
  const size_t samples = n < 16 ? n : 16;
  for (size_t k = 0; k < samples; k++) {
    const size_t i = samples == 1 ? 0 : k * (n - 1) / (samples - 1);
    const uint8_t* r = (const uint8_t*)host + i * rec_bytes;
    for (size_t b = 0; b < rec_bytes; b++) h = (h ^ r[b]) * 1099511628211ull;
  }
  return h;
}

// Base cache (ecg_msm_ex cache_bases): entries keyed by (host pointer, n,
// curve, layout) and a fingerprint of sampled records.  A hit returns the
// entry's prepared buffer; a same-key entry with other content is dropped.
static void* cache_find(ecg_ctx* ctx, const void* bases, size_t n, int curve_id, int layout, uint64_t fp) {
  for (size_t k = 0; k < ctx->base_cache.size(); k++) {
    auto& e = ctx->base_cache[k];
    if (e.host == bases && e.n == n && e.curve == curve_id && e.layout == layout) {
      if (e.fingerprint == fp) return e.dev;
      (void)hipStreamSynchronize(ctx->stream);  // same address, other content: drop the stale entry
      base_cache_release(e.dev);
      ctx->base_cache.erase(ctx->base_cache.begin() + k);
      return nullptr;
    }
  }
  return nullptr;
}

static void cache_insert(ecg_ctx* ctx, const void* bases, size_t n, int curve_id, int layout, void* dev,
                         uint64_t fp) {
  if (ctx->base_cache.size() >= 8) {  // bounded: drop the oldest entry
    (void)hipStreamSynchronize(ctx->stream);
    base_cache_release(ctx->base_cache.front().dev);
    ctx->base_cache.erase(ctx->base_cache.begin());
  }
  ctx->base_cache.push_back({bases, n, curve_id, layout, dev, fp});
}

static size_t host_rec_bytes(int curve_id, int layout) {
  const size_t lq = fq_limbs64(curve_id);
  return layout == ECG_BASES_ARK_AFFINE ? (2 * lq + 1) * 8 : 2 * lq * 8;
}

// Bases on the device for (bases, layout, n).  Uncached: uploaded (and
// converted from the ark layout) into the workspace slot `slot` as [x, y].
// Cached: kept as a prepared buffer (msm_prepare_run: the records the bucket
// kernels gather), so a cache hit runs as a prepared MSM; the [x, y] staging
// copy is released after the conversion.
static int stage_bases(ecg_ctx* ctx, int curve_id, const void* bases, int layout, size_t n, int cache,
                       const char* slot, void** d_out) {
  const size_t lq = fq_limbs64(curve_id);
  const size_t xy_bytes = n * 2 * lq * 8;
  const size_t rec = host_rec_bytes(curve_id, layout);
  hipStream_t s = ctx->stream;
  uint64_t fp = 0;
  if (cache) {
    fp = bases_fingerprint(bases, n, rec);
    if (void* hit = cache_find(ctx, bases, n, curve_id, layout, fp)) {
      *d_out = hit;
      return ECG_OK;
    }
  }
  const char* xy_slot = cache ? "cache_stage_xy" : slot;
  void* xy;
  ECG_TRY(ws_get(ctx, xy_slot, xy_bytes, &xy));
  if (n) {
    if (layout == ECG_BASES_ARK_AFFINE) {
      void* raw;
      ECG_TRY(ws_get(ctx, "prep_ark_raw", n * rec, &raw));
      ECG_HIP(hipMemcpyAsync(raw, bases, n * rec, hipMemcpyHostToDevice, s));
      ECG_TRY(bases_from_ark(ctx, curve_id, raw, n, xy, s));
    } else {
      ECG_HIP(hipMemcpyAsync(xy, bases, xy_bytes, hipMemcpyHostToDevice, s));
    }
  }
  if (!cache) {
    *d_out = xy;
    return ECG_OK;
  }
  void* prep = nullptr;
  ECG_TRY(msm_prepare_run(ctx, curve_id, xy, n, 0, &prep, s));  // synchronises s
  ws_release(ctx, "cache_stage_xy");
  ws_release(ctx, "prep_ark_raw");
  cache_insert(ctx, bases, n, curve_id, layout, prep, fp);
  *d_out = prep;
  return ECG_OK;
}

// Cached bases and host exponents of at least this many terms: the exponents
// go up in passes overlapped with the previous pass's compute (msm_host_run).
constexpr size_t MSMX_PIPE_MIN = (size_t)1 << 22;

int ecg_msm_ex(ecg_ctx* ctx, int curve_id, const void* bases, int bases_layout, size_t n_bases, size_t skip,
               const uint64_t* exps, int exps_montgomery, size_t n_exps, const uint64_t* density, int cache_bases,
               uint64_t* out_jac, ecg_abort_cb abort_cb, void* user) {
  ECG_ENTER(ctx);
  if (!out_jac || (n_exps && !exps) || (n_bases && !bases)) {
    set_error("ecg_msm_ex: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!curve_valid(curve_id)) {
    set_error("multiexp: unknown curve_id %d", curve_id);
    return ECG_ERR_INVALID;
  }
  if (bases_layout != ECG_BASES_XY && bases_layout != ECG_BASES_ARK_AFFINE) {
    set_error("ecg_msm_ex: unknown bases_layout %d", bases_layout);
    return ECG_ERR_INVALID;
  }
  hipStream_t s = ctx->stream;
  if (cache_bases && !density && n_exps >= MSMX_PIPE_MIN) {
    // resident bases: only the exponents travel, pass by pass behind the compute
    if (skip > n_bases || n_exps > n_bases - skip) {
      set_error("Expected more bases from source.");  // multiexp_cpu.rs:55-61
      return ECG_ERR_INVALID;
    }
    const uint64_t fp = bases_fingerprint(bases, n_bases, host_rec_bytes(curve_id, bases_layout));
    void* d_prep = cache_find(ctx, bases, n_bases, curve_id, bases_layout, fp);
    if (!d_prep && skip == 0 && n_exps == n_bases) {
      // cold: the entry is filled pass by pass inside the pipelined MSM (the
      // base uploads overlap the compute instead of preceding it)
      ECG_TRY(msm_prepared_alloc(ctx, curve_id, n_bases, 0, &d_prep, s));
      const MsmFill fill{bases, bases_layout == ECG_BASES_ARK_AFFINE, curve_id};
      int rc = msm_host_run(ctx, curve_id, d_prep, 1, exps, n_exps, exps_montgomery, out_jac, abort_cb, user, &fill);
      (void)hipStreamSynchronize(s);
      if (rc != ECG_OK) {
        msm_prepared_free(d_prep);  // partly filled: never cached
        return rc;
      }
      cache_insert(ctx, bases, n_bases, curve_id, bases_layout, d_prep, fp);
      return kt_collect(ctx);
    }
    if (!d_prep) ECG_TRY(stage_bases(ctx, curve_id, bases, bases_layout, n_bases, 1, nullptr, &d_prep));
    const uint8_t* b0 = (const uint8_t*)d_prep + skip * msm_prepared_stride(curve_id, 0);
    int rc = msm_host_run(ctx, curve_id, b0, 1, exps, n_exps, exps_montgomery, out_jac, abort_cb, user);
    (void)hipStreamSynchronize(s);
    if (rc != ECG_OK) return rc;
    return kt_collect(ctx);
  }
  // exps -> device, density-compacted on device (generate_exps)
  void *d_e, *d_ec;
  ECG_TRY(ws_get(ctx, "msmx_exps", n_exps * 32, &d_e));
  if (n_exps) ECG_HIP(hipMemcpyAsync(d_e, exps, n_exps * 32, hipMemcpyHostToDevice, s));
  size_t dense = n_exps;
  d_ec = d_e;
  if (density) {
    void* d_bits;
    const size_t nw = (n_exps + 63) / 64;
    ECG_TRY(ws_get(ctx, "msmx_bits", nw * 8, &d_bits));
    if (nw) ECG_HIP(hipMemcpyAsync(d_bits, density, nw * 8, hipMemcpyHostToDevice, s));
    ECG_TRY(ws_get(ctx, "msmx_exps_dense", n_exps * 32, &d_ec));
    ECG_TRY(density_compact(ctx, d_e, (const uint64_t*)d_bits, n_exps, d_ec, &dense, s));
  }
  if (skip > n_bases || dense > n_bases - skip) {
    set_error("Expected more bases from source.");  // multiexp_cpu.rs:55-61
    return ECG_ERR_INVALID;
  }
  // bases: the whole (cached) array, or just the [skip, skip + dense) window
  const size_t lq = fq_limbs64(curve_id);
  void* d_xy;
  const uint8_t* d_base0;
  if (cache_bases) {  // a prepared buffer: base-aligned offset in its record stride
    ECG_TRY(stage_bases(ctx, curve_id, bases, bases_layout, n_bases, 1, nullptr, &d_xy));
    d_base0 = (const uint8_t*)d_xy + skip * msm_prepared_stride(curve_id, 0);
  } else {
    const size_t rec = bases_layout == ECG_BASES_ARK_AFFINE ? (2 * lq + 1) * 8 : 2 * lq * 8;
    ECG_TRY(stage_bases(ctx, curve_id, (const uint8_t*)bases + skip * rec, bases_layout, dense, 0, "msmx_bases",
                        &d_xy));
    d_base0 = (const uint8_t*)d_xy;
  }
  int rc = msm_run(ctx, curve_id, d_base0, d_ec, dense, out_jac, s, abort_cb, user, exps_montgomery);
  (void)hipStreamSynchronize(s);
  if (rc != ECG_OK) return rc;
  return kt_collect(ctx);
}

int ecg_point_sum_dev(ecg_ctx* ctx, int curve_id, const void* d_points, size_t count, uint64_t* out_jac,
                      void* stream) {
  ECG_ENTER(ctx);
  if (!out_jac || (!d_points && count)) {
    set_error("ecg_point_sum_dev: null pointer");
    return ECG_ERR_INVALID;
  }
  return point_sum_run(ctx, curve_id, d_points, count, out_jac, pick_stream(ctx, stream));
}

// ---------------------------------------------------------------- device buffers
int ecg_dev_alloc(ecg_ctx* ctx, size_t bytes, void** out) {
  ECG_ENTER(ctx);
  if (!out) {
    set_error("ecg_dev_alloc: null out pointer");
    return ECG_ERR_INVALID;
  }
  hipError_t e = hipMalloc(out, bytes ? bytes : 16);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("device allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    *out = nullptr;
    return ECG_ERR_NOMEM;
  }
  return ECG_OK;
}

void ecg_dev_free(ecg_ctx* ctx, void* p) {
  if (!ctx || !p) return;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  // a prepared-bases buffer (from any context) is unregistered with its memory
  if (!msm_prepared_free(p)) (void)hipFree(p);
}

int ecg_dev_upload(ecg_ctx* ctx, void* d_dst, const void* src, size_t bytes) {
  ECG_ENTER(ctx);
  ECG_HIP(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return ECG_OK;
}

int ecg_dev_download(ecg_ctx* ctx, void* dst, const void* d_src, size_t bytes) {
  ECG_ENTER(ctx);
  ECG_HIP(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ECG_HIP(hipStreamSynchronize(ctx->stream));
  return ECG_OK;
}

int ecg_msm_multi(ecg_ctx** ctxs, int nctx, int curve_id, const uint64_t* bases_xy, const uint64_t* scalars,
                  size_t n, uint64_t* out_jac, ecg_abort_cb abort_cb, void* user) {
  if (!ctxs || nctx <= 0) {
    set_error("No working GPUs found!");
    return ECG_ERR_NODEV;
  }
  if (!out_jac) {
    set_error("ecg_msm_multi: null output");
    return ECG_ERR_INVALID;
  }
  const size_t lq = fq_limbs64(curve_id);
  const size_t chunk = nctx > 0 ? (n + nctx - 1) / nctx : n;  // multiexp.rs:332-336
  std::vector<uint64_t> partials((size_t)nctx * 3 * lq, 0);
  std::atomic<int> first_err{ECG_OK};
  std::mutex mu;
  std::string err_msg;
  std::vector<std::thread> th;
  // every worker polls this before each device pass: the caller's abort, or
  // another worker's error (first error wins, multiexp.rs:354-359)
  struct Poll {
    ecg_abort_cb cb;
    void* user;
    std::atomic<int>* first_err;
    static int fn(void* p) {
      const Poll* q = (const Poll*)p;
      return q->first_err->load() != ECG_OK || (q->cb && q->cb(q->user)) ? 1 : 0;
    }
  } poll{abort_cb, user, &first_err};
  int used = 0;
  for (int d = 0; d < nctx; d++) {
    const size_t i0 = std::min(n, d * chunk), i1 = std::min(n, i0 + chunk);
    if (d > 0 && i0 >= i1) break;
    used++;
    th.emplace_back([&, d, i0, i1]() {
      int rc = msm_host(ctxs[d], curve_id, bases_xy + i0 * 2 * lq, scalars + i0 * 4, i1 - i0,
                        partials.data() + (size_t)d * 3 * lq, &Poll::fn, &poll);
      if (rc != ECG_OK) {
        int expected = ECG_OK;
        if (first_err.compare_exchange_strong(expected, rc)) {
          std::lock_guard<std::mutex> g(mu);
          err_msg = g_err;
        }
      }
    });
  }
  for (auto& t : th) t.join();
  if (first_err.load() != ECG_OK) {
    g_err = err_msg;
    return first_err.load();
  }
  if (used == 1) {
    memcpy(out_jac, partials.data(), 3 * lq * 8);
    return ECG_OK;
  }
  // cross-device fold of the per-device partials (multiexp.rs:394-397)
  return point_sum_host(curve_id, partials.data(), used, out_jac);
}

int ecg_point_sum(int curve_id, const uint64_t* points, size_t count, uint64_t* out_jac) {
  if (!out_jac || (!points && count)) {
    set_error("ecg_point_sum: null pointer");
    return ECG_ERR_INVALID;
  }
  return point_sum_host(curve_id, points, count, out_jac);
}

int ecg_msm_check_bases(int curve_id, const uint64_t* bases_xy, const uint64_t* scalars, size_t n) {
  const size_t lq = fq_limbs64(curve_id);
  for (size_t i = 0; i < n; i++) {
    const uint64_t* e = scalars + 4 * i;
    if ((e[0] | e[1] | e[2] | e[3]) == 0) continue;
    uint64_t o = 0;
    for (size_t k = 0; k < 2 * lq; k++) o |= bases_xy[i * 2 * lq + k];
    if (o == 0) {
      set_error("Encountered an identity element in the CRS.");
      return ECG_ERR_INVALID;
    }
  }
  return ECG_OK;
}

int ecg_gen_bases_dev(ecg_ctx* ctx, int curve_id, const uint64_t* a, const uint64_t* b, size_t n, void* d_out,
                      void* stream) {
  ECG_ENTER(ctx);
  if (!a || !b || (!d_out && n)) {
    set_error("ecg_gen_bases_dev: null pointer");
    return ECG_ERR_INVALID;
  }
  if (!(b[0] | b[1] | b[2] | b[3])) {  // the generator steps by bG: b = 0 would step by the identity
    set_error("ecg_gen_bases_dev: b must be non-zero (the bases step by b G; upload equal bases instead)");
    return ECG_ERR_INVALID;
  }
  return gen_bases_run(ctx, curve_id, a, b, n, d_out, pick_stream(ctx, stream));
}

int ecg_ctx_set_mem_limit(ecg_ctx* ctx, size_t bytes) {
  ECG_ENTER(ctx);
  ctx->mem_limit = bytes;
  return ECG_OK;
}

int ecg_ctx_release_workspace(ecg_ctx* ctx) {
  ECG_ENTER(ctx);
  // queued work on any stream may still use a buffer (pick_stream): drain the device
  ECG_HIP(hipDeviceSynchronize());
  for (auto& kv : ctx->ws)
    if (kv.second.ptr) ECG_HIP(hipFree(kv.second.ptr));
  ctx->ws.clear();
  ctx->tw_fid = -1;  // the NTT's twiddle tables lived in the workspace
  return ECG_OK;
}

int ecg_ctx_set_msm_chunk(ecg_ctx* ctx, size_t max_terms) {
  ECG_ENTER(ctx);
  if (max_terms > 0x7fffffffull) {
    set_error("ecg_ctx_set_msm_chunk: at most 2^31-1 terms per pass");
    return ECG_ERR_INVALID;
  }
  ctx->msm_chunk = max_terms;
  return ECG_OK;
}

int ecg_msm_chunk_size(ecg_ctx* ctx, int curve_id, size_t* out) {
  ECG_ENTER(ctx);
  if (!out) {
    set_error("ecg_msm_chunk_size: null pointer");
    return ECG_ERR_INVALID;
  }
  return msm_pass_terms_run(ctx, curve_id, out);
}

const char* ecg_runtime_info(void) {
  static std::string info;
  static std::once_flag once;
  std::call_once(once, [] {
    int hv = 0, nv = 0;
    (void)hipRuntimeGetVersion(&hv);
    (void)ncclGetVersion(&nv);
    Dl_info dh{}, dn{};
    (void)dladdr(reinterpret_cast<void*>(&hipRuntimeGetVersion), &dh);
    (void)dladdr(reinterpret_cast<void*>(&ncclGetVersion), &dn);
    char buf[1024];
    snprintf(buf, sizeof buf, "hip=%d (%s); rccl=%d (%s)", hv, dh.dli_fname ? dh.dli_fname : "?", nv,
             dn.dli_fname ? dn.dli_fname : "?");
    info = buf;
  });
  return info.c_str();
}

int ecg_last_kernel_time(ecg_ctx* ctx, const char* name, double* ms_total, int* launches) {
  if (!ctx || !name) {
    set_error("ecg_last_kernel_time: null pointer");
    return ECG_ERR_INVALID;
  }
  auto it = ctx->ktimes.find(name);
  if (it == ctx->ktimes.end()) {
    if (ms_total) *ms_total = 0;
    if (launches) *launches = 0;
    return ECG_OK;
  }
  if (ms_total) *ms_total = it->second.ms;
  if (launches) *launches = it->second.launches;
  return ECG_OK;
}

}  // extern "C"
