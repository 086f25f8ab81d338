// curve_id dispatch of the MSM drivers.  The per-curve kernels and drivers
// (msm_impl.hpp) are compiled once per curve in msm_inst.hip (-DECG_INST=id),
// which exports one MsmOps table each; this file only routes calls.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
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

// ---------------------------------------------------------------------------
// Prepared-bases registry (ecg_msm_prepare_bases / _table).  Process-wide,
// keyed by the data's address range, so a prepared buffer is recognised from
// any context on its device and through any base-aligned pointer into it
// (e.g. one rank's shard handed to ecg_msm_dist).  Each allocation starts
// with a header (magic + a per-buffer nonce) in front of the records: a
// buffer released behind the library's back (hipFree of some other pointer
// cannot be seen) and reused by a new allocation no longer carries its
// nonce, so a stale entry is detected and dropped instead of its memory
// being read as records.
// ---------------------------------------------------------------------------
namespace {
constexpr size_t PREP_HEADER = 256;  // keeps the records 256-B aligned
constexpr uint64_t PREP_MAGIC = 0x3150455250474345ull;  // "ECGPREP1"
struct PrepEntry {
  int device;
  int curve;
  size_t n;         // bases
  uint32_t tab_c;   // > 0: window table (ecg_msm_prepare_table)
  size_t stride;    // bytes per base (all of its table rows)
  uint64_t nonce;
};
std::mutex g_prep_mu;
std::map<uintptr_t, PrepEntry> g_prep;  // records' start address -> entry
std::atomic<uint64_t> g_prep_seq{0x9E3779B97F4A7C15ull};
}  // namespace

// The header check of a prepared buffer, deferred into the call's stream:
// prep_check_kernel compares the header with the entry's magic and nonce and
// writes the verdict into mapped pinned host memory, which the caller reads
// once the call has synchronised (prepared_confirm).  A synchronous 16-B
// hipMemcpy of the header before every call cost ~0.2 ms of host-side latency
// (profiles/r05/msm_2p20_timeline_pinned_d2h.txt: the copy blit 0.2 ms after
// the previous call's last kernel), 5 % of a 2^20 MSM.
struct PrepCheck {
  bool pending = false;
  uintptr_t start = 0;
  uint64_t nonce = 0;
  volatile uint32_t* flag = nullptr;  // 0 = not run, 1 = ours, 2 = stale
};

__global__ void prep_check_kernel(const uint64_t* __restrict__ hdr, uint64_t magic, uint64_t nonce,
                                  uint32_t* __restrict__ flag) {
  if (threadIdx.x == 0) flag[0] = (hdr[0] == magic && hdr[1] == nonce) ? 1u : 2u;
}

static void prepared_drop(uintptr_t start, uint64_t nonce) {  // freed outside the library
  std::lock_guard<std::mutex> g(g_prep_mu);
  auto it = g_prep.find(start);
  if (it != g_prep.end() && it->second.nonce == nonce) g_prep.erase(it);
}

// After the stream has synchronised: true if the deferred check found the
// buffer's own header (or nothing was deferred); false drops the stale entry.
static bool prepared_confirm(const PrepCheck& chk) {
  if (!chk.pending) return true;
  if (*chk.flag == 1u) return true;
  prepared_drop(chk.start, chk.nonce);
  return false;
}

// Is d_bases inside a prepared buffer?  It must then sit on a base boundary,
// on ctx's device, and cover the n bases the call reads, for the same curve.
// With `defer` (and a stream), the header is checked on the stream instead of
// by a synchronous copy; the caller must then call prepared_confirm after its
// work has synchronised and redo the call as unprepared if it returns false.
static int prepared_lookup(ecg_ctx* ctx, int curve_id, const void* d_bases, size_t n, const char* what,
                           BaseForm* bf, hipStream_t s = nullptr, PrepCheck* defer = nullptr) {
  *bf = BaseForm{};
  if (defer) *defer = PrepCheck{};
  const uintptr_t a = (uintptr_t)d_bases;
  PrepEntry e;
  uintptr_t start;
  {
    std::lock_guard<std::mutex> g(g_prep_mu);
    auto it = g_prep.upper_bound(a);
    if (it == g_prep.begin()) return ECG_OK;
    --it;
    if (a >= it->first + it->second.n * it->second.stride && !(it->second.n == 0 && a == it->first)) return ECG_OK;
    start = it->first;
    e = it->second;
  }
  // still our allocation?  The header is read only while header and records
  // still lie inside one live device allocation (a released range may be
  // unmapped, or reused by an allocation that starts elsewhere); then it must
  // carry this buffer's magic and nonce.
  uint64_t hdr[2] = {0, 0};
  hipDeviceptr_t alloc_base = nullptr;
  size_t alloc_size = 0;
  const uintptr_t h0 = start - PREP_HEADER, h1 = start + e.n * e.stride;
  const bool live = hipMemGetAddressRange(&alloc_base, &alloc_size, (hipDeviceptr_t)h0) == hipSuccess &&
                    (uintptr_t)alloc_base <= h0 && h1 <= (uintptr_t)alloc_base + alloc_size;
  if (!live) {
    (void)hipGetLastError();
    prepared_drop(start, e.nonce);
    return ECG_OK;
  }
  if (defer && e.device == ctx->device) {  // header checked on the stream (prep_check_kernel)
    void *h_flag, *d_flag;
    ECG_TRY(hws_get(ctx, "prep_check", 16, &h_flag, &d_flag));
    *(volatile uint32_t*)h_flag = 0u;
    hipLaunchKernelGGL(prep_check_kernel, dim3(1), dim3(64), 0, s, (const uint64_t*)(start - PREP_HEADER),
                       PREP_MAGIC, e.nonce, (uint32_t*)d_flag);
    ECG_HIP(hipGetLastError());
    *defer = PrepCheck{true, start, e.nonce, (volatile uint32_t*)h_flag};
  } else if (hipMemcpy(hdr, (const void*)(start - PREP_HEADER), sizeof hdr, hipMemcpyDeviceToHost) != hipSuccess ||
             hdr[0] != PREP_MAGIC || hdr[1] != e.nonce) {
    (void)hipGetLastError();
    prepared_drop(start, e.nonce);
    return ECG_OK;
  }
  // a refusal of a deferred entry waits for its header check first: a stale
  // entry (the address now holds someone else's [x, y] bases) is dropped and
  // the call goes on unprepared, instead of refusing every later call
  auto refuse = [&]() -> int {
    if (defer && defer->pending) {
      (void)hipStreamSynchronize(s);
      if (!prepared_confirm(*defer)) {
        *defer = PrepCheck{};
        (void)hipGetLastError();
        return ECG_OK;
      }
    }
    return ECG_ERR_INVALID;
  };
  if (e.device != ctx->device) {
    set_error("%s: the prepared bases live on device %d, the context is on device %d", what, e.device, ctx->device);
    return ECG_ERR_INVALID;
  }
  const size_t off = a - start;
  if (off % e.stride) {
    set_error("%s: pointer %zu bytes into prepared bases is not on a base boundary (%zu bytes per base)", what, off,
              e.stride);
    return refuse();
  }
  const size_t avail = e.n - off / e.stride;
  if (e.curve != curve_id || n > avail) {
    set_error("%s: prepared bases hold %zu bases of curve %d from this pointer, the call reads %zu of curve %d", what,
              avail, e.curve, n, curve_id);
    return refuse();
  }
  bf->prepared = true;
  bf->tab_c = e.tab_c;
  bf->tab_n = avail;
  return ECG_OK;
}

bool msm_prepared_free(void* p) {
  std::lock_guard<std::mutex> g(g_prep_mu);
  auto it = g_prep.find((uintptr_t)p);
  if (it == g_prep.end()) return false;
  const uint64_t zero[2] = {0, 0};  // retire the header: a later lookup of a reused address cannot match
  (void)hipMemcpy((char*)p - PREP_HEADER, zero, sizeof zero, hipMemcpyHostToDevice);
  (void)hipFree((char*)p - PREP_HEADER);
  (void)hipGetLastError();
  g_prep.erase(it);
  return true;
}

size_t msm_prepared_stride(int curve_id, uint32_t tab_c) {
  const MsmOps* o = msm_ops(curve_id, "prepared_stride");
  if (!o) return 0;
  if (!tab_c) return o->record_bytes();
  const uint32_t W = tab_c >= 2 && tab_c <= 25 ? o->table_windows(tab_c) : 0u;
  return W ? o->record_bytes() * W : 0;
}

int msm_plan_info_run(int curve_id, size_t n, uint32_t window_bits, uint32_t* c, uint32_t* windows, int* sort_mode) {
  const MsmOps* o = msm_ops(curve_id, "plan_info");
  if (!o) return ECG_ERR_INVALID;
  if (window_bits > 22) {
    set_error("plan_info: window_bits %u out of range [0, 22] (0 = automatic)", window_bits);
    return ECG_ERR_INVALID;
  }
  return o->plan_info(n, window_bits, c, windows, sort_mode);
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
  PrepCheck chk;
  ECG_TRY(prepared_lookup(ctx, curve_id, d_bases, n, "multiexp", &bf, s, &chk));
  int rc = o->single(ctx, d_bases, d_scalars, n, out_jac, s, abort_cb, user, scalar_mont != 0, bf);
  (void)hipStreamSynchronize(s);
  // released behind the library's back: not our records (on every return path,
  // so a failed first run still drops the stale entry)
  if (!prepared_confirm(chk))
    rc = o->single(ctx, d_bases, d_scalars, n, out_jac, s, abort_cb, user, scalar_mont != 0, BaseForm{});
  return rc;
}

int msm_grid_run(ecg_ctx* ctx, int curve_id, const void* d_bases, const void* d_scalars, size_t n, int rank,
                 int nranks, uint64_t* out_jac, hipStream_t s, ecg_abort_cb abort_cb, void* user, int* pieces) {
  if (pieces) *pieces = 0;
  if (n > 0x7fffffffull) {
    set_error("multiexp: at most 2^31-1 terms per call");
    return ECG_ERR_INVALID;
  }
  if (nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("msm_dist_grid: rank %d of %d", rank, nranks);
    return ECG_ERR_INVALID;
  }
  const MsmOps* o = msm_ops(curve_id, "multiexp");
  if (!o) return ECG_ERR_INVALID;
  uint32_t c = 0, W = 0;
  int mode = 0;
  ECG_TRY(o->plan_info(n ? n : 1, 0, &c, &W, &mode));
  BaseForm bf;
  PrepCheck chk;
  ECG_TRY(prepared_lookup(ctx, curve_id, d_bases, n, "multiexp", &bf, s, &chk));
  if (bf.tab_c) {
    (void)hipStreamSynchronize(s);
    if (prepared_confirm(chk)) {
      set_error("msm_dist_grid: the bases are a window table; the grid split needs plain prepared or [x, y] bases");
      return ECG_ERR_INVALID;
    }
    bf = BaseForm{};  // a stale table entry: the pointer holds [x, y] bases
    chk = PrepCheck{};
  }
  const size_t lq = fq_limbs64(curve_id);
  // grid entries e = w n + t (window-major); this rank's range [a, b)
  const unsigned __int128 T = (unsigned __int128)W * n;
  const uint64_t a = (uint64_t)(T * (unsigned)rank / (unsigned)nranks);
  const uint64_t b = (uint64_t)(T * (unsigned)(rank + 1) / (unsigned)nranks);
  // one core call over the rank's window blocks (msm_grid_t); ECG_MSM_GRID_PIECES=1 runs the
  // former piece-by-piece form (A/B)
  static const bool by_pieces = [] {
    const char* e = getenv("ECG_MSM_GRID_PIECES");
    return e && e[0] == '1';
  }();
  // (a share of more than 16 windows -- small n, few ranks -- runs piece by piece)
  const bool one_call = !by_pieces && (a >= b || (b - 1) / n - a / n + 1 <= 16);
  auto run = [&](BaseForm f) -> int {
    if (one_call) {
      if (a >= b) {  // no grid cell for this rank (more ranks than cells): the identity
        if (pieces) *pieces = 0;
        return o->point_sum(nullptr, 0, out_jac);
      }
      // Entries one device pass may hold: the terms per pass of a whole MSM (msm_pass_terms,
      // calc_chunk_size's memory budget, multiexp.rs:71-93) times its windows.  A larger share
      // (huge n, or a context capped by ecg_ctx_set_mem_limit / ecg_ctx_set_msm_chunk) runs as
      // consecutive sub-ranges of the grid, one core call each, whose partials are summed.
      const uint64_t max_e = std::max<uint64_t>((uint64_t)o->pass_terms(ctx) * W, 1);
      std::vector<uint64_t> parts;
      int np = 0;
      for (uint64_t e0 = a; e0 < b;) {
        uint64_t e1 = std::min<uint64_t>(b, e0 + max_e);
        const uint32_t w0 = (uint32_t)(e0 / n);
        if ((e1 - 1) / n - w0 + 1 > 16) e1 = (uint64_t)(w0 + 16) * n;  // at most 16 window blocks per call
        const uint32_t wl = (uint32_t)((e1 - 1) / n);
        if (abort_cb && abort_cb(user)) return ECG_ABORTED;  // multiexp.rs:140-144, per device pass
        parts.resize(parts.size() + 3 * lq);
        ECG_TRY(o->grid(ctx, d_bases, d_scalars, n, w0, wl - w0 + 1, (size_t)(e0 - (uint64_t)w0 * n),
                        (size_t)(e1 - (uint64_t)wl * n), parts.data() + parts.size() - 3 * lq, s, f));
        np++;
        e0 = e1;
      }
      if (pieces) *pieces = np;
      if (np == 1) {
        memcpy(out_jac, parts.data(), 3 * lq * 8);
        return ECG_OK;
      }
      return o->point_sum(parts.data(), (size_t)np, out_jac);
    }
    const size_t stride = f.prepared ? msm_prepared_stride(curve_id, 0) : 2 * lq * 8;
    std::vector<uint64_t> parts;
    int np = 0;
    uint64_t e = a;
    while (e < b) {
      if (abort_cb && abort_cb(user)) return ECG_ABORTED;  // multiexp.rs:140-144, per device pass
      const uint32_t w = (uint32_t)(e / n);
      const size_t t0 = (size_t)(e - (uint64_t)w * n);
      uint32_t nwin = 1;
      size_t t1 = n;
      if (t0 == 0) {  // whole windows run as one piece (one core call, W = nwin groups)
        nwin = (uint32_t)((b - e) / n);
        if (nwin == 0) {
          nwin = 1;
          t1 = (size_t)(b - e);
        }
      } else if (b - (uint64_t)w * n < n) {
        t1 = (size_t)(b - (uint64_t)w * n);
      }
      parts.resize(parts.size() + 3 * lq);
      ECG_TRY(o->piece(ctx, (const uint8_t*)d_bases + t0 * stride, (const uint8_t*)d_scalars + t0 * 32, t1 - t0, n,
                       w, nwin, parts.data() + parts.size() - 3 * lq, s, f));
      np++;
      e = (uint64_t)(w + nwin - 1) * n + t1;
    }
    if (pieces) *pieces = np;
    return o->point_sum(parts.data(), (size_t)np, out_jac);
  };
  int rc = run(bf);
  (void)hipStreamSynchronize(s);
  if (!prepared_confirm(chk)) rc = run(BaseForm{});  // stale: the pointer holds [x, y] bases
  return rc;
}

uint32_t msm_table_window_auto(int curve_id, size_t n) {
  const MsmOps* o = msm_ops(curve_id, "prepare_table");
  return o ? o->table_auto(n) : 0;
}

// A registered prepared buffer of n bases (plain records) whose records the
// caller fills on stream s before anything reads them (msm_host_t's cold
// cache fill); released with msm_prepared_free.
int msm_prepared_alloc(ecg_ctx* ctx, int curve_id, size_t n, uint32_t tab_c, void** d_out, hipStream_t s) {
  const MsmOps* o = msm_ops(curve_id, "prepare_bases");
  if (!o) return ECG_ERR_INVALID;
  const size_t bytes = o->prepared_bytes(n, tab_c);
  void* base = nullptr;
  hipError_t e = hipMalloc(&base, bytes + PREP_HEADER);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("prepare_bases: device allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return ECG_ERR_NOMEM;
  }
  void* p = (char*)base + PREP_HEADER;
  const uint64_t nonce = g_prep_seq.fetch_add(0x9E3779B97F4A7C15ull) ^ (uint64_t)(uintptr_t)p;
  const uint64_t hdr[2] = {PREP_MAGIC, nonce};
  if (hipMemcpyAsync(base, hdr, sizeof hdr, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    set_error("prepare_bases: %s", hipGetErrorString(hipGetLastError()));
    (void)hipFree(base);
    return ECG_ERR_HIP;
  }
  const size_t stride = o->record_bytes() * (tab_c ? o->table_windows(tab_c) : 1u);
  {
    std::lock_guard<std::mutex> g(g_prep_mu);
    g_prep[(uintptr_t)p] = PrepEntry{ctx->device, curve_id, n, tab_c, stride, nonce};
  }
  *d_out = p;
  return ECG_OK;
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
  void* p = nullptr;
  ECG_TRY(msm_prepared_alloc(ctx, curve_id, n, tab_c, &p, s));
  int rc = o->prepare(ctx, d_bases, n, tab_c, p, s);
  if (rc == ECG_OK && hipStreamSynchronize(s) != hipSuccess) {
    set_error("prepare_bases: %s", hipGetErrorString(hipGetLastError()));
    rc = ECG_ERR_HIP;
  }
  if (rc != ECG_OK) {
    msm_prepared_free(p);
    return rc;
  }
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
  PrepCheck chk;
  ECG_TRY(prepared_lookup(ctx, curve_id, d_bases, n_bases, "multiple_multiexp", &bf, s, &chk));
  int rc = o->batch(ctx, d_bases, d_scalars, (uint32_t)n_lines, (uint32_t)n_chunks, line_len, scalar_mont != 0,
                    window_bits, out_jac, s, bf);
  (void)hipStreamSynchronize(s);
  if (!prepared_confirm(chk))  // released behind the library's back: not our records
    rc = o->batch(ctx, d_bases, d_scalars, (uint32_t)n_lines, (uint32_t)n_chunks, line_len, scalar_mont != 0,
                  window_bits, out_jac, s, BaseForm{});
  return rc;
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

int msm_host_run(ecg_ctx* ctx, int curve_id, const void* bases, int bases_resident, const void* h_scalars, size_t n,
                 int scalar_mont, uint64_t* out_jac, ecg_abort_cb abort_cb, void* user, const MsmFill* fill) {
  if (n > 0x7fffffffull) {
    set_error("multiexp: at most 2^31-1 terms per call");
    return ECG_ERR_INVALID;
  }
  const MsmOps* o = msm_ops(curve_id, "multiexp");
  if (!o) return ECG_ERR_INVALID;
  BaseForm bf;
  if (bases_resident) {  // must be (a base-aligned view into) a prepared buffer
    ECG_TRY(prepared_lookup(ctx, curve_id, bases, n, "multiexp", &bf));
    if (!bf.prepared) {
      set_error("multiexp: resident bases must be a prepared buffer");
      return ECG_ERR_INVALID;
    }
  }
  if (fill && (!bf.prepared || bf.tab_c)) {
    set_error("multiexp: a cache fill needs a plain prepared buffer");
    return ECG_ERR_INVALID;
  }
  return o->host(ctx, bases, bf, h_scalars, n, scalar_mont ? 1u : 0u, out_jac, abort_cb, user, fill);
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
