/*
 * ecgpu.h -- C ABI of the MI355X-native MSM + radix-FFT engine (libecgpu.so).
 *
 * This is the drop-in boundary for the reference's ec-gpu-gen host API
 * (kriptohaberciniz/0g-ec-gpu, crate ec-gpu-proxy).  A thin binding (the Rust
 * shim in INTEGRATION.md, or the Python mirror in 0g-ec-gpu_amd/ecgpu/) keeps
 * the reference's types and calls these functions; no rust-gpu-tools, no
 * CUDA/OpenCL dispatch.  Signatures use plain pointers and sizes only.
 *
 * Element layouts are exactly the arkworks 0.4 in-memory layouts the
 * reference passes around:
 *   field element  : N little-endian u64 limbs, Montgomery form, R = 2^(64N),
 *                    fully reduced (ark_ff::Fp<MontBackend<_,N>,N>);
 *                    Fr: N = 4 (32 B); BLS12-381 Fq: N = 6 (48 B); BN254 Fq: N = 4.
 *   scalar (exp)   : BigInt<4>, canonical little-endian u64 limbs (32 B)
 *                    (PrimeFieldRepr::to_bigint, ag-types/src/impls.rs:7-18).
 *   base           : [x, y] Montgomery, identity = all zero
 *                    (GpuRepr::to_gpu_repr, ag-types/src/impls.rs:48-58).
 *                    G2 coordinates are Fq2 = [c0, c1] (QuadExtField), so a
 *                    coordinate is Lq = 2 x (Fq limbs): 12 u64 for BLS12-381
 *                    G2, 8 for BN254 G2.
 *   result point   : Jacobian [X, Y, Z] Montgomery (G::Curve), normalised:
 *                    (x, y, 1) or the identity (0, 1, 0).
 *
 * Return codes: 0 = ok, 1 = aborted (EcError::Aborted), < 0 = error
 * (EcError::Simple / GpuTools); ecg_last_error() gives the thread's message.
 * All calls are synchronous and thread-safe for distinct contexts.
 */
#ifndef ECGPU_H
#define ECGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ids ------------------------------------------------------------- */
#define ECG_FIELD_BLS12_381_FR 0
#define ECG_FIELD_BLS12_381_FQ 1
#define ECG_FIELD_BN254_FR 2
#define ECG_FIELD_BN254_FQ 3

#define ECG_CURVE_BLS12_381 0 /* G1 over BLS12-381 Fq, scalars in Fr */
#define ECG_CURVE_BN254 1     /* G1 over BN254 Fq, scalars in Fr      */
#define ECG_CURVE_BLS12_381_G2 2 /* G2 over BLS12-381 Fq2 (field2.cl), scalars in Fr */
#define ECG_CURVE_BN254_G2 3     /* G2 over BN254 Fq2, scalars in Fr               */

#define ECG_OK 0
#define ECG_ABORTED 1
#define ECG_ERR_INVALID (-1)  /* bad argument (EcError::Simple)            */
#define ECG_ERR_HIP (-2)      /* HIP runtime error (EcError::GpuTools)     */
#define ECG_ERR_NOMEM (-3)    /* device allocation failed                  */
#define ECG_ERR_NODEV (-4)    /* "No working GPUs found!"                  */
#define ECG_ERR_RCCL (-5)     /* collective failed                         */

/* Polled between FFT passes / MSM chunks; non-zero => abort
 * (the reference's maybe_abort: &dyn Fn() -> bool, fft.rs:94-98,
 * multiexp.rs:140-144). */
typedef int (*ecg_abort_cb)(void *user);

typedef struct ecg_ctx ecg_ctx;

/* ---- devices and contexts ---------------------------------------------
 * Replace rust_gpu_tools::Device::all() + ec_gpu_program::program!(device)
 * (ec-gpu-program/src/program.rs:11-29, 97-106).  A context owns one HIP
 * device, one stream and a grow-only device workspace (twiddle tables,
 * MSM bucket arrays) that persists across calls. */
int ecg_device_count(void);
int ecg_ctx_create(int device, ecg_ctx **out);
void ecg_ctx_destroy(ecg_ctx *ctx);
/* device memory and compute units (Device::memory / compute_units,
 * used by multiexp.rs:109-127) */
int ecg_ctx_info(ecg_ctx *ctx, size_t *mem_bytes, int *compute_units);
/* Wait for all work on ctx's device (bench barriers). */
int ecg_ctx_synchronize(ecg_ctx *ctx);
/* MSM terms per device pass -- SingleMultiexpKernel::n as calc_chunk_size
 * derives it from Device::memory (multiexp.rs:71-93,109-127): the engine's
 * per-term workspace against (1 - MEMORY_PADDING) of the device memory minus
 * the resident base cache, and at most the device's free memory at the call
 * plus the context's own MSM buffers (so buffers the caller keeps resident,
 * other contexts and other processes shrink it).  Longer MSMs run as several passes, the abort
 * callback polled before each (multiexp.rs:140-144,348-361).
 * ecg_ctx_set_msm_chunk pins it (1 .. 2^31-1; 0 restores the derived value). */
int ecg_msm_chunk_size(ecg_ctx *ctx, int curve_id, size_t *out_terms);
int ecg_ctx_set_msm_chunk(ecg_ctx *ctx, size_t max_terms);
/* Cap the device memory this context plans with and allocates as scratch
 * (bytes; 0 = the device's memory): calc_chunk_size's pass sizing uses it,
 * and a scratch allocation that would take the context's workspace past it
 * fails with ECG_ERR_NOMEM.  For ranks or provers that share one GPU, as the
 * reference's MEMORY_PADDING leaves room for other users (multiexp.rs:24). */
int ecg_ctx_set_mem_limit(ecg_ctx *ctx, size_t bytes);
/* Free the context's device workspace (the grow-only scratch of its MSMs,
 * NTTs and EC-FFTs, and the cached twiddle tables) after draining the device;
 * the next call regrows what it needs.  The reference frees its buffers when
 * a Program / CudaWorkspace is dropped (ag-cuda-proxy/src/module.rs:23-42);
 * here a long-lived context hands the memory back without being destroyed,
 * e.g. before one transform that needs most of the 288 GB (a 2^32 NTT: data
 * plus scratch, 275 GB).  Prepared bases, the base cache and device buffers
 * the caller allocated are not touched. */
int ecg_ctx_release_workspace(ecg_ctx *ctx);
/* "hip=<version> (<libamdhip64 path>); rccl=<version> (<librccl path>)": the
 * HIP runtime and RCCL this process actually bound (launchers check it is the
 * ROCm install's, not another copy loaded earlier into the process). */
const char *ecg_runtime_info(void);
const char *ecg_last_error(void);
const char *ecg_version(void);
/* rust_gpu_tools::Device's queries for one device without a context
 * (Device::name / memory / compute_units, used by multiexp.rs:109-127):
 * name gets the marketing name and gfx arch, NUL-terminated in name_cap bytes. */
int ecg_device_info(int device, size_t *mem_bytes, int *compute_units, char *name, size_t name_cap);

/* ---- kernel registry --------------------------------------------------------
 * The HIP kernels are compiled into this library ahead of time, so the
 * reference's build-time code generator (ag_build::SourceBuilder::{add_field,
 * add_fft, add_ec, add_ec_fft, add_multiexp} + generate, ag-build/src/
 * source/builder.rs:43-99, lib.rs:47-53) becomes a query of which
 * instantiations the library holds.  Fields and curves are named by their
 * moduli, exactly what ag_types::GpuField::modulus() / ark_ff::Field::
 * characteristic() report (ag-types/src/lib.rs:33-50), so a generic kernel
 * needs no extra trait bound to find its id.  Moduli are little-endian u64
 * limbs (high zero limbs ignored); degree is the extension degree over the
 * prime field (1, or 2 for the G2 coordinate field Fq2). */
#define ECG_FIELD_BLS12_381_FQ2 4 /* registry only: add_field::<Fq2>  */
#define ECG_FIELD_BN254_FQ2 5
#define ECG_KIND_FIELD 0    /* add_field    -> field id  */
#define ECG_KIND_FFT 1      /* add_fft      -> field id  */
#define ECG_KIND_EC 2       /* add_ec       -> curve id  */
#define ECG_KIND_EC_FFT 3   /* add_ec_fft   -> curve id  */
#define ECG_KIND_MULTIEXP 4 /* add_multiexp -> curve id  */
/* field id, or ECG_ERR_INVALID (last error names the modulus) */
int ecg_field_id(const uint64_t *modulus, size_t limbs, uint32_t degree);
/* curve id from the coordinate field (base_degree 1 = G1, 2 = G2) and the
 * scalar field, or ECG_ERR_INVALID */
int ecg_curve_id(const uint64_t *base_modulus, size_t base_limbs, uint32_t base_degree,
                 const uint64_t *scalar_modulus, size_t scalar_limbs);
/* 1 if the library holds kernels of `kind` for id (a field id for FIELD/FFT,
 * a curve id otherwise), else 0 */
int ecg_has_kernel(int kind, int id);
/* "bls12_381_fr", "bn254_g2", ...; NULL for an unknown id */
const char *ecg_field_name(int field_id);
const char *ecg_curve_name(int curve_id);

/* ---- FFT ----------------------------------------------------------------
 * In-place forward DFT of size 2^log_n over field_id (an Fr), natural order
 * in and out, no 1/n scaling: a[k] <- sum_j a[j] * omega^(j k).
 * Replaces SingleFftKernel::radix_fft (ec-gpu-proxy/src/fft.rs:50-135) and
 * FftKernel::radix_fft (fft.rs:200-204).  log_n = 0 is rejected
 * (the reference panics, fft.rs:68-70); log_n <= the field's 2-adicity. */
int ecg_fft(ecg_ctx *ctx, int field_id, uint64_t *inout, const uint64_t *omega, uint32_t log_n,
            ecg_abort_cb abort_cb, void *user);

/* FftKernel::radix_fft_many (fft.rs:211-246): `count` transforms
 * distributed in ceil(count / nctx) chunks, one host thread per context,
 * first error wins. */
int ecg_fft_many(ecg_ctx **ctxs, int nctx, int field_id, uint64_t **inouts, const uint64_t *omegas,
                 const uint32_t *log_ns, size_t count, ecg_abort_cb abort_cb, void *user);

/* Device-resident variant: d_inout is a device pointer on ctx's device
 * (n x 32 B); `stream` is a hipStream_t (NULL = the context's stream).
 * Inputs stay in HBM; used by bench.py and by callers that keep
 * polynomials resident. */
int ecg_fft_dev(ecg_ctx *ctx, int field_id, void *d_inout, const uint64_t *omega, uint32_t log_n,
                void *stream);

/* ---- EC-FFT (FFT over G1, "FFTg") -------------------------------------------
 * In-place DFT of 2^log_n G1 points: P_k <- sum_j omega^(j k) * P_j, natural
 * order in and out, omega an Fr element (Montgomery, 4 x u64) that is a
 * primitive 2^log_n-th root of unity.  inout: 2^log_n Jacobian points
 * (3 x Lq u64 each, any Z; Z = 0 is the identity), rewritten normalised.
 * Replaces SingleEcFftKernel::radix_ec_fft (ec-gpu-proxy/src/ec_fft.rs:56-164)
 * and ag_cuda_ec::ec_fft::radix_ec_fft (ag-cuda-ec/src/ec_fft.rs:12-93);
 * result == serial_ec_fft (ec_fft_cpu.rs:12-56).  log_n <= min(31, Fr
 * two-adicity); log_n = 0 returns the (normalised) input. */
int ecg_ec_fft(ecg_ctx *ctx, int curve_id, uint64_t *inout_jac, const uint64_t *omega, uint32_t log_n,
               ecg_abort_cb abort_cb, void *user);
/* Largest radix (as log2) of the EC-FFT stages, process-wide: 1 = radix-2
 * stages only, up to 8; 0 (default) = the engine's choice per size (radix-2^d
 * stages for the small, latency-bound transforms).  Results
 * never depend on it.  A/B and test knob, as ECG_ECFFT_RADIX. */
int ecg_ec_fft_set_radix(int max_log_radix);
/* EcFftKernel::radix_ec_fft_many (ec_fft.rs:224-270): ceil(count / nctx)
 * transforms per context, one host thread per context, first error wins. */
int ecg_ec_fft_many(ecg_ctx **ctxs, int nctx, int curve_id, uint64_t **inouts, const uint64_t *omegas,
                    const uint32_t *log_ns, size_t count, ecg_abort_cb abort_cb, void *user);
/* Device-resident variant (d_inout_jac on ctx's device). */
int ecg_ec_fft_dev(ecg_ctx *ctx, int curve_id, void *d_inout_jac, const uint64_t *omega, uint32_t log_n,
                   void *stream);

/* ---- MSM ------------------------------------------------------------------
 * out = sum_{i<n} scalars[i] * bases[i] on curve_id's G1.
 * Replaces SingleMultiexpKernel::multiexp (ec-gpu-proxy/src/multiexp.rs:135-236)
 * and MultiexpKernel::multiexp (multiexp.rs:372-400, called with
 * bases + skip already applied).  Identity bases contribute nothing (the
 * reference CPU path rejects them, multiexp_cpu.rs:57-61; use
 * ecg_msm_check_bases to reproduce that error).  Any 256-bit scalar is
 * accepted and reduced mod r (same group element as multiexp_cpu). */
int ecg_msm(ecg_ctx *ctx, int curve_id, const uint64_t *bases_xy, const uint64_t *scalars, size_t n,
            uint64_t *out_jac, ecg_abort_cb abort_cb, void *user);

/* MultiexpKernel::parallel_multiexp + multiexp (multiexp.rs:324-400):
 * contiguous ceil(n / nctx) ranges, one host thread per context, each range
 * in device passes of at most ecg_msm_chunk_size terms, first error wins
 * (every worker polls it before each of its passes, as it polls abort_cb, and
 * stops with the first error), partial sums folded on the
 * host (multiexp.rs:394-397).  A context listed twice is used by one thread
 * at a time (every call holds its context's lock). */
int ecg_msm_multi(ecg_ctx **ctxs, int nctx, int curve_id, const uint64_t *bases_xy,
                  const uint64_t *scalars, size_t n, uint64_t *out_jac, ecg_abort_cb abort_cb,
                  void *user);

/* Device-resident variant (cf. ag_cuda_ec::multiexp::upload_multiexp_bases,
 * ag-cuda-ec/src/multiexp.rs:11-19): d_bases / d_scalars are device
 * pointers on ctx's device.  out_jac is host memory (3 x Lq u64) or, with
 * out_on_device != 0, a device pointer. */
int ecg_msm_dev(ecg_ctx *ctx, int curve_id, const void *d_bases, const void *d_scalars, size_t n,
                void *out_jac, int out_on_device, void *stream);

/* upload_multiexp_bases (ag-cuda-ec/src/multiexp.rs:11-19) in the engine's
 * own layout: converts n device-resident [x, y] bases (d_bases, as
 * ecg_msm_dev takes them) ONCE into a new device buffer in the layout the
 * bucket kernels gather (G1: 128-B reduced-radix records; G2: [x, y]) and
 * returns it in *d_prepared.  Pass *d_prepared as d_bases to ecg_msm_dev,
 * ecg_multiple_multiexp or ecg_msm_dist (any call reading at most n bases of
 * the same curve): those calls then skip the per-call conversion.  A
 * pointer k records into the buffer (k x the per-base record size, e.g. a
 * rank's shard) reads bases k.. in the same form; a pointer inside it that
 * is not on a record boundary is refused.  The buffer belongs to its device,
 * not to ctx: any context on that device may use it.  It is immutable
 * (re-prepare after changing the bases); release it with ecg_dev_free (on
 * any context) -- never with hipFree. */
int ecg_msm_prepare_bases(ecg_ctx *ctx, int curve_id, const void *d_bases, size_t n, void **d_prepared);
/* Bytes per base in a prepared buffer (window_bits = 0: plain records;
 * else the window table of that window size): the stride of base-aligned
 * pointers into it.  0 for an unknown curve or a table form the curve lacks. */
size_t ecg_msm_prepared_stride(int curve_id, uint32_t window_bits);

/* Fixed-base form of ecg_msm_prepare_bases for bases reused across many
 * MSMs (upload_multiexp_bases's use in ag-cuda-ec, multiexp.rs:11-19): also
 * precomputes the window table 2^(k c) P_i for the W = ceil(256 / c) windows
 * (c = window_bits; 0 = chosen for an n-term MSM: 24 at 2^26).  MSMs over
 * the returned buffer put every window's digit into ONE bucket set, which
 * removes the per-window bucket reduction and admits a larger window (fewer
 * mixed adds per term).  Same results as any other base form.  Memory: W x
 * the prepared records (2^26 BLS12-381 bases at c = 24: 11 x 8 GiB).
 * G1 curves only; W x n < 2^31.  Use and release as ecg_msm_prepare_bases. */
int ecg_msm_prepare_table(ecg_ctx *ctx, int curve_id, const void *d_bases, size_t n, uint32_t window_bits,
                          void **d_prepared);

/* The window size ecg_msm_prepare_table picks (window_bits = 0) for MSMs of
 * n terms -- for multiple_multiexp pass the chunk length.  0 for curves
 * without a table form (G2) or an unknown curve_id. */
uint32_t ecg_msm_table_window(int curve_id, size_t n);

/* Batched multi-line MSM: ag_cuda_ec::multiexp::multiple_multiexp
 * (ag-cuda-ec/src/multiexp.rs:21-81; kernel ag-build/cl/multiexp.cl:215-262).
 * d_bases holds n_bases affine points (x, y Montgomery, identity = zeros) as
 * uploaded by upload_multiexp_bases (multiexp.rs:11-19), i.e. n_bases /
 * line_len lines of line_len bases; `scalars` is ONE row of line_len canonical
 * scalars (4 x u64 each) shared by every line -- host memory, or device memory
 * with scalars_on_device != 0.  Each line is split into num_chunks chunks of
 * line_len / num_chunks terms (a remainder is ignored, as the reference's
 * kernel does) and out_jac[line * num_chunks + chunk] (3 x Lq u64, host
 * memory, normalised Jacobian) receives that chunk's MSM.  window_bits = 0
 * lets the engine choose the window; 1..22 pins it (the reference's
 * window_size; results never depend on it).  The reference's neg_is_cheap
 * flag has no analogue: digits are always signed. */
int ecg_multiple_multiexp(ecg_ctx *ctx, int curve_id, const void *d_bases, size_t n_bases,
                          const uint64_t *scalars, int scalars_on_device, int scalars_montgomery,
                          size_t line_len, size_t num_chunks, uint32_t window_bits,
                          uint64_t *out_jac);

/* ---- MSM with the reference's host-side prep done on device --
 *   bases_layout ECG_BASES_XY          : [x, y] GpuRepr records (2 x Lq u64)
 *                ECG_BASES_ARK_AFFINE  : arkworks Affine {x, y, infinity: bool}
 *                                        records (2 x Lq u64 + 8 B), converted
 *                                        on device (ag-types/src/impls.rs:48-58)
 *   exps_montgomery != 0 : exps are Fr elements in Montgomery form; to_bigint
 *                          (impls.rs:13) runs in the digit kernel
 *   density != NULL      : bitmap of n_exps bits (bitvec Lsb0, u64 words); only
 *                          exps with a set bit take part, consuming bases in
 *                          order from `skip` -- DensityTracker::generate_exps
 *                          (multiexp_cpu.rs:127-138) compacted on device, then
 *                          MultiexpKernel::multiexp(bases, exps, skip)
 *                          (multiexp.rs:372-400)
 *   cache_bases != 0     : keep the converted bases resident, keyed by
 *                          (bases pointer, n_bases, curve, layout); later calls
 *                          with the same key skip the upload (the caller must
 *                          not mutate the array; ecg_base_cache_clear drops it)
 * Too few bases for the dense exps -> ECG_ERR_INVALID "Expected more bases
 * from source." (multiexp_cpu.rs:55-61). */
#define ECG_BASES_XY 0
#define ECG_BASES_ARK_AFFINE 1
int ecg_msm_ex(ecg_ctx *ctx, int curve_id, const void *bases, int bases_layout, size_t n_bases,
               size_t skip, const uint64_t *exps, int exps_montgomery, size_t n_exps,
               const uint64_t *density, int cache_bases, uint64_t *out_jac, ecg_abort_cb abort_cb,
               void *user);
void ecg_base_cache_clear(ecg_ctx *ctx);
/* Host addresses of the bases arrays currently held by ctx's base cache
 * (at most 8 entries, oldest first; the oldest is evicted by a new one):
 * writes up to cap of them to out and returns how many are cached.  Lets a
 * binding release its references to arrays the cache no longer holds. */
size_t ecg_base_cache_keys(ecg_ctx *ctx, const void **out, size_t cap);

/* The plan of a one-task MSM of n terms on curve_id -- ecg_msm_dev's
 * (window_bits = 0) or ecg_multiple_multiexp's with num_chunks = 1 and the
 * window pinned to window_bits: window bits c, windows W = ceil((|r| + 1) / c)
 * and how the per-window bucket entries are sorted.  Not in the reference
 * API: tests use it to assert which pipeline branch a case exercises. */
#define ECG_SORT_GLOBAL 0   /* one sort over (group, bucket) keys            */
#define ECG_SORT_PW_ONE 1   /* window-padded blocks, one sort over all blocks */
#define ECG_SORT_PW_BLOCK 2 /* window-padded blocks, one sort per block      */
int ecg_msm_plan_info(int curve_id, size_t n, uint32_t window_bits, uint32_t *c, uint32_t *windows,
                      int *sort_mode);

/* Element-wise field operations on the device, one engine field form at a
 * time: the reference's GPU field tests (ag-build/src/tests/test_fields.rs:
 * test_add/sub/mul/pow/sqr/double/mont/unmont over field.cl:14-392).
 * form 0 = boundary form (field.hpp); 1 = the product path's reduced-radix
 * form (fieldrr.hpp: Fr 9 x 29, BLS12-381 Fq 13 x 30, BN254 Fq 9 x 29);
 * 2 = an Fq's second reduced-radix form (BLS12-381 14 x 29, BN254 10 x 28: the
 * G2 components).  a, b, out: n elements of host memory in the field's
 * Montgomery form (ECG_FOP_MONT takes canonical inputs, ECG_FOP_UNMONT returns
 * them; forms 1-2 have neither); e is ECG_FOP_POW's exponent; b may be NULL
 * for the unary ops.  Outputs are canonical (fully reduced). */
#define ECG_FOP_ADD 0
#define ECG_FOP_SUB 1
#define ECG_FOP_MUL 2
#define ECG_FOP_SQR 3
#define ECG_FOP_DOUBLE 4
#define ECG_FOP_POW 5
#define ECG_FOP_MONT 6
#define ECG_FOP_UNMONT 7
#define ECG_FOP_INV 8
int ecg_field_ops(ecg_ctx *ctx, int field_id, int form, int op, const uint64_t *a, const uint64_t *b, uint32_t e,
                  size_t n, uint64_t *out);

/* Sum `count` Jacobian points (3 x Lq u64 each, device memory) into one
 * normalised Jacobian point: the EC fold that follows the RCCL all-gather of
 * per-GPU partials (RCCL has no EC-add reduction op).  The points are copied
 * to the host and folded there (a few adds); out is host memory. */
int ecg_point_sum_dev(ecg_ctx *ctx, int curve_id, const void *d_points, size_t count,
                      uint64_t *out_jac, void *stream);
/* Same fold over host memory (multiexp.rs:394-397 cross-device sum). */
int ecg_point_sum(int curve_id, const uint64_t *points, size_t count, uint64_t *out_jac);

/* Returns ECG_ERR_INVALID with "Encountered an identity element in the
 * CRS." if any base with a non-zero scalar is the identity -- the
 * reference CPU path's error behaviour (multiexp_cpu.rs:57-61). */
int ecg_msm_check_bases(int curve_id, const uint64_t *bases_xy, const uint64_t *scalars, size_t n);

/* ---- multi-GPU over RCCL (one process per GPU) ------------------
 * Replace the reference's host-thread-per-device dispatch (multiexp.rs:324-367,
 * fft.rs:211-246) for the one-process-per-GPU launch: rank 0 makes a 128-byte
 * id, the launcher broadcasts it, every rank calls ecg_comm_init on its own
 * context.  nranks = 1 with a NULL id: no communicator (exchanges become
 * device copies); with an id: a real one-rank RCCL communicator.
 *
 * Failure semantics (the reference stops every device at the first error,
 * multiexp.rs:345-365, fft.rs:218-245): the distributed calls exchange every
 * rank's status before their payload collectives, so a rank that fails
 * locally (bad argument, allocation, abort_cb) makes EVERY rank return an
 * error instead of leaving its peers blocked in a collective: the lowest
 * failing rank's code (ECG_ABORTED stays ECG_ABORTED), with the local message
 * on that rank and "rank k failed" on the others.  The communicator is
 * non-blocking: initialisation and every collective wait under a deadline
 * (ecg_comm_set_timeout; default ECG_COMM_TIMEOUT_S or 300 s), after which
 * the communicator is aborted and the call returns ECG_ERR_RCCL (a peer that
 * crashed or never arrived).  An aborted communicator, or one whose
 * ecg_comm_init failed, refuses later distributed calls until ecg_comm_init
 * runs again.  The status records travel through staging reserved at
 * ecg_comm_init, so no allocation can keep a failed rank out of the status
 * exchange. */
int ecg_comm_unique_id(uint8_t *out /* 128 bytes */);
/* What the context's communicator reports: rank count, this rank and its HIP
 * device (ncclCommCount / ncclCommUserRank / ncclCommCuDevice for RCCL; the
 * init arguments for the host transport), the device's PCI bus id
 * (NUL-terminated, bus_cap bytes, may be NULL) and the transport. */
#define ECG_COMM_NONE 0   /* one rank, no communicator */
#define ECG_COMM_RCCL 1
#define ECG_COMM_HOST 2
#define ECG_COMM_FAILED 3 /* several ranks, communicator aborted or never up */
int ecg_comm_info(ecg_ctx *ctx, int *nranks, int *rank, int *device, char *bus_id, size_t bus_cap,
                  int *transport);
/* Wall time (us) of the last ecg_msm_dist's status + partial exchange. */
int ecg_comm_last_exchange(ecg_ctx *ctx, double *us);
int ecg_comm_init(ecg_ctx *ctx, int nranks, int rank, const uint8_t *unique_id);
void ecg_comm_destroy(ecg_ctx *ctx);
/* Deadline of communicator initialisation and of each exchange, in ms
 * (0 = ECG_COMM_TIMEOUT_S or 300 s).  Applies to the next ecg_comm_init too. */
int ecg_comm_set_timeout(ecg_ctx *ctx, uint32_t ms);
/* Host transport instead of RCCL: the caller's launcher group moves the
 * bytes (e.g. ranks that share a GPU, which RCCL refuses, or a launcher that
 * already holds an MPI / gloo group).  xchg(op, send, recv, bytes, user)
 * returns 0 on success:
 *   ECG_XCHG_ALLGATHER: send = bytes, recv = nranks x bytes in rank order;
 *   ECG_XCHG_ALLTOALL : send = nranks x bytes (block q goes to rank q),
 *                       recv = nranks x bytes (block q came from rank q).
 * Buffers are host memory; the callback runs on the calling thread. */
#define ECG_XCHG_ALLGATHER 0
#define ECG_XCHG_ALLTOALL 1
typedef int (*ecg_xchg_cb)(int op, const void *send, void *recv, size_t bytes, void *user);
int ecg_comm_init_host(ecg_ctx *ctx, int nranks, int rank, ecg_xchg_cb xchg, void *user);
/* RCCL all-gather / equal-split all-to-all of device buffers (synchronous). */
int ecg_comm_allgather(ecg_ctx *ctx, const void *d_send, void *d_recv, size_t bytes);
int ecg_comm_alltoall(ecg_ctx *ctx, const void *d_send, void *d_recv, size_t bytes_per_peer);
/* MSM over this rank's contiguous shard (multiexp.rs:332-336 split); the
 * per-rank partial points are all-gathered over RCCL and folded on the host
 * (multiexp.rs:394-397; RCCL has no EC-add reduction), so every rank gets
 * the full result in out_jac (host, 3 x Lq u64).  Each rank's status rides
 * in the same all-gather as its partial (one collective per call). */
int ecg_msm_dist(ecg_ctx *ctx, int curve_id, const void *d_bases, const void *d_scalars, size_t n_local,
                 uint64_t *out_jac);
/* With the reference's maybe_abort (multiexp.rs:140-144): polled before each
 * device pass of the local MSM; an abort on any rank returns ECG_ABORTED on
 * every rank. */
int ecg_msm_dist_ex(ecg_ctx *ctx, int curve_id, const void *d_bases, const void *d_scalars, size_t n_local,
                    uint64_t *out_jac, ecg_abort_cb abort_cb, void *user);
/* Grid split of the same MSM (SURVEY §8(e)'s window partitioning with
 * replicated bases): every rank passes ALL n bases and scalars; the n-term
 * plan's (window x term) grid is cut into nranks equal ranges of W n / nranks
 * cells and rank r runs the r-th (a partial window, whole windows, a partial
 * window: at most three Pippenger pieces, each with the whole-n plan's window
 * width), so every rank does the same bucket work whatever n and nranks are.
 * Partials and statuses are exchanged and folded as in ecg_msm_dist; the
 * result is bit-identical to ecg_msm over the n terms.  Bases may be a
 * prepared buffer (ecg_msm_prepare) or [x, y] records, not a window table.
 * Every rank must pass the same n: n rides in the status record, and ranks
 * called with different sizes all return ECG_ERR_INVALID.  A share larger
 * than one device pass (the context's memory budget, ecg_ctx_set_mem_limit /
 * ecg_ctx_set_msm_chunk) runs as several passes. */
int ecg_msm_dist_grid(ecg_ctx *ctx, int curve_id, const void *d_bases, const void *d_scalars, size_t n,
                      uint64_t *out_jac);
int ecg_msm_dist_grid_ex(ecg_ctx *ctx, int curve_id, const void *d_bases, const void *d_scalars, size_t n,
                         uint64_t *out_jac, ecg_abort_cb abort_cb, void *user);
/* Rank `rank` of `nranks`'s local step of ecg_msm_dist_grid on this context,
 * without an exchange: its partial (normalised Jacobian) in out_jac and, if
 * pieces is not NULL, the number of Pippenger pieces it ran. */
int ecg_msm_grid_part(ecg_ctx *ctx, int curve_id, const void *d_bases, const void *d_scalars, size_t n, int rank,
                      int nranks, uint64_t *out_jac, int *pieces);
/* One NTT of 2^log_n points, block-distributed (rank r holds points
 * [r m, (r+1) m), m = 2^log_n / nranks), in place, natural order: the
 * four-step split of parallel_fft (fft_cpu.rs:59-111) with three RCCL
 * all-to-alls.  nranks a power of two <= 16, 2^log_n >= 2 nranks^2.
 * Statuses are exchanged before the first all-to-all and after the local
 * NTT (abort_cb polled at both, as fft.rs:94-98 polls it per pass). */
int ecg_fft_dist(ecg_ctx *ctx, int field_id, void *d_local, const uint64_t *omega, uint32_t log_n);
int ecg_fft_dist_ex(ecg_ctx *ctx, int field_id, void *d_local, const uint64_t *omega, uint32_t log_n,
                    ecg_abort_cb abort_cb, void *user);
/* Its local steps (for callers that drive the exchanges themselves):
 * stage1: T-point DFT across the received segments + twiddle; stage3: the
 * final [T][m/T] -> [m/T][T] interleave.  See dfft.hip for the layouts. */
int ecg_fft_dist_stage1(ecg_ctx *ctx, int field_id, const void *d_in, void *d_out, const uint64_t *omega,
                        uint32_t nranks, uint32_t rank, uint32_t log_n);
int ecg_fft_dist_stage3(ecg_ctx *ctx, const void *d_in, void *d_out, uint32_t nranks, uint32_t log_n);

/* ---- device buffers on ctx's device ---------------------------------------
 * Keep bases / polynomials resident in HBM across calls: the analogue of
 * ag_cuda_ec::multiexp::upload_multiexp_bases and ag-cuda-proxy's
 * DeviceData::upload (ag-cuda-ec/src/multiexp.rs:11-19,
 * ag-cuda-proxy/src/params.rs:112-219).  Pointers feed the *_dev calls. */
int ecg_dev_alloc(ecg_ctx *ctx, size_t bytes, void **out);
void ecg_dev_free(ecg_ctx *ctx, void *d_ptr);
int ecg_dev_upload(ecg_ctx *ctx, void *d_dst, const void *src, size_t bytes);
int ecg_dev_download(ecg_ctx *ctx, void *dst, const void *d_src, size_t bytes);

/* ---- synthetic inputs for benchmarks/tests (not part of the reference API)
 * Bases P_i = (a + i*b) * G for i < n written to device memory d_out
 * (n x 2 x Lq u64, GpuRepr layout); a, b canonical 4-limb scalars, b != 0
 * (ECG_ERR_INVALID otherwise: the generator steps by b G). */
int ecg_gen_bases_dev(ecg_ctx *ctx, int curve_id, const uint64_t *a, const uint64_t *b, size_t n,
                      void *d_out, void *stream);

/* Kernel timing of the most recent call on this context (ms per launch of
 * the dominant kernel, and its launch count), recorded with HIP events on
 * the stream the kernels ran on.  name is "ntt_pass" or "msm_accumulate". */
int ecg_last_kernel_time(ecg_ctx *ctx, const char *name, double *ms_total, int *launches);

#ifdef __cplusplus
}
#endif
#endif /* ECGPU_H */
