//! Raw bindings to libecgpu.so: one `extern "C"` declaration per entry point of
//! `include/ecgpu.h`, same order, same argument meaning.  The replacement
//! crates of this workspace (rust-gpu-tools, ec-gpu-program, ag-build, the
//! ec-gpu-proxy `amd` modules, ag-cuda-ec) wrap it in the reference's types.
//! `tests/test_rust_shim.py` checks this file against the header (names,
//! arity, pointer/scalar kinds, constants) so the two cannot drift.

use std::os::raw::{c_char, c_int, c_void};

// ---- ids (ECG_FIELD_* / ECG_CURVE_*) -------------------------------------
pub const ECG_FIELD_BLS12_381_FR: c_int = 0;
pub const ECG_FIELD_BLS12_381_FQ: c_int = 1;
pub const ECG_FIELD_BN254_FR: c_int = 2;
pub const ECG_FIELD_BN254_FQ: c_int = 3;

pub const ECG_CURVE_BLS12_381: c_int = 0;
pub const ECG_CURVE_BN254: c_int = 1;
pub const ECG_CURVE_BLS12_381_G2: c_int = 2;
pub const ECG_CURVE_BN254_G2: c_int = 3;

// ---- kernel registry (ag_build::SourceBuilder kinds) ------------------------
pub const ECG_FIELD_BLS12_381_FQ2: c_int = 4;
pub const ECG_FIELD_BN254_FQ2: c_int = 5;
pub const ECG_KIND_FIELD: c_int = 0;
pub const ECG_KIND_FFT: c_int = 1;
pub const ECG_KIND_EC: c_int = 2;
pub const ECG_KIND_EC_FFT: c_int = 3;
pub const ECG_KIND_MULTIEXP: c_int = 4;

// ---- return codes -----------------------------------------------------------
pub const ECG_OK: c_int = 0;
pub const ECG_ABORTED: c_int = 1;
pub const ECG_ERR_INVALID: c_int = -1;
pub const ECG_ERR_HIP: c_int = -2;
pub const ECG_ERR_NOMEM: c_int = -3;
pub const ECG_ERR_NODEV: c_int = -4;
pub const ECG_ERR_RCCL: c_int = -5;

// ---- ecg_msm_ex base layouts --------------------------------------------------
pub const ECG_BASES_XY: c_int = 0;
pub const ECG_BASES_ARK_AFFINE: c_int = 1;

// ---- ecg_msm_plan_info sort modes ---------------------------------------------
pub const ECG_FOP_ADD: c_int = 0;
pub const ECG_FOP_SUB: c_int = 1;
pub const ECG_FOP_MUL: c_int = 2;
pub const ECG_FOP_SQR: c_int = 3;
pub const ECG_FOP_DOUBLE: c_int = 4;
pub const ECG_FOP_POW: c_int = 5;
pub const ECG_FOP_MONT: c_int = 6;
pub const ECG_FOP_UNMONT: c_int = 7;
pub const ECG_FOP_INV: c_int = 8;
pub const ECG_SORT_GLOBAL: c_int = 0;
pub const ECG_SORT_PW_ONE: c_int = 1;
pub const ECG_SORT_PW_BLOCK: c_int = 2;

/// `typedef int (*ecg_abort_cb)(void *user)`: polled between FFT passes and
/// MSM device passes (the reference's `maybe_abort`, fft.rs:94-98,
/// multiexp.rs:140-144).
pub type ecg_abort_cb = Option<unsafe extern "C" fn(user: *mut c_void) -> c_int>;

// ---- host transport ops (ecg_comm_init_host) -----------------------------------
pub const ECG_XCHG_ALLGATHER: c_int = 0;
pub const ECG_XCHG_ALLTOALL: c_int = 1;
// ecg_comm_info transports
pub const ECG_COMM_NONE: c_int = 0;
pub const ECG_COMM_RCCL: c_int = 1;
pub const ECG_COMM_HOST: c_int = 2;
pub const ECG_COMM_FAILED: c_int = 3;

/// `typedef int (*ecg_xchg_cb)(int op, const void *send, void *recv, size_t
/// bytes, void *user)`: the launcher's group moves the exchange bytes
/// (host memory) instead of RCCL; returns 0 on success.
pub type ecg_xchg_cb =
    Option<unsafe extern "C" fn(op: c_int, send: *const c_void, recv: *mut c_void, bytes: usize,
                                user: *mut c_void) -> c_int>;

/// Opaque `ecg_ctx`: one device, one stream, a grow-only workspace, a lock.
#[repr(C)]
pub struct ecg_ctx {
    _private: [u8; 0],
}

#[link(name = "ecgpu")]
extern "C" {
    // ---- devices and contexts (program.rs:11-29, 97-106) ----
    pub fn ecg_device_count() -> c_int;
    pub fn ecg_ctx_create(device: c_int, out: *mut *mut ecg_ctx) -> c_int;
    pub fn ecg_ctx_destroy(ctx: *mut ecg_ctx);
    pub fn ecg_ctx_info(ctx: *mut ecg_ctx, mem_bytes: *mut usize, compute_units: *mut c_int) -> c_int;
    pub fn ecg_ctx_synchronize(ctx: *mut ecg_ctx) -> c_int;
    pub fn ecg_msm_chunk_size(ctx: *mut ecg_ctx, curve_id: c_int, out_terms: *mut usize) -> c_int;
    pub fn ecg_ctx_set_msm_chunk(ctx: *mut ecg_ctx, max_terms: usize) -> c_int;
    pub fn ecg_ctx_set_mem_limit(ctx: *mut ecg_ctx, bytes: usize) -> c_int;
    pub fn ecg_ctx_release_workspace(ctx: *mut ecg_ctx) -> c_int;
    pub fn ecg_runtime_info() -> *const c_char;
    pub fn ecg_last_error() -> *const c_char;
    pub fn ecg_version() -> *const c_char;
    pub fn ecg_device_info(device: c_int, mem_bytes: *mut usize, compute_units: *mut c_int, name: *mut c_char,
                           name_cap: usize) -> c_int;

    // ---- kernel registry (ag-build/src/source/builder.rs:43-99, lib.rs:47-53) ----
    pub fn ecg_field_id(modulus: *const u64, limbs: usize, degree: u32) -> c_int;
    pub fn ecg_curve_id(base_modulus: *const u64, base_limbs: usize, base_degree: u32,
                        scalar_modulus: *const u64, scalar_limbs: usize) -> c_int;
    pub fn ecg_has_kernel(kind: c_int, id: c_int) -> c_int;
    pub fn ecg_field_name(field_id: c_int) -> *const c_char;
    pub fn ecg_curve_name(curve_id: c_int) -> *const c_char;

    // ---- FFT (fft.rs:50-135, 200-246) ----
    pub fn ecg_fft(ctx: *mut ecg_ctx, field_id: c_int, inout: *mut u64, omega: *const u64, log_n: u32,
                   abort_cb: ecg_abort_cb, user: *mut c_void) -> c_int;
    pub fn ecg_fft_many(ctxs: *mut *mut ecg_ctx, nctx: c_int, field_id: c_int, inouts: *mut *mut u64,
                        omegas: *const u64, log_ns: *const u32, count: usize, abort_cb: ecg_abort_cb,
                        user: *mut c_void) -> c_int;
    pub fn ecg_fft_dev(ctx: *mut ecg_ctx, field_id: c_int, d_inout: *mut c_void, omega: *const u64,
                       log_n: u32, stream: *mut c_void) -> c_int;

    // ---- EC-FFT (ec_fft.rs:56-164, 224-270) ----
    pub fn ecg_ec_fft(ctx: *mut ecg_ctx, curve_id: c_int, inout_jac: *mut u64, omega: *const u64, log_n: u32,
                      abort_cb: ecg_abort_cb, user: *mut c_void) -> c_int;
    pub fn ecg_ec_fft_set_radix(max_log_radix: c_int) -> c_int;
    pub fn ecg_ec_fft_many(ctxs: *mut *mut ecg_ctx, nctx: c_int, curve_id: c_int, inouts: *mut *mut u64,
                           omegas: *const u64, log_ns: *const u32, count: usize, abort_cb: ecg_abort_cb,
                           user: *mut c_void) -> c_int;
    pub fn ecg_ec_fft_dev(ctx: *mut ecg_ctx, curve_id: c_int, d_inout_jac: *mut c_void, omega: *const u64,
                          log_n: u32, stream: *mut c_void) -> c_int;

    // ---- MSM (multiexp.rs:135-236, 324-400; ag-cuda-ec/src/multiexp.rs:11-81) ----
    pub fn ecg_msm(ctx: *mut ecg_ctx, curve_id: c_int, bases_xy: *const u64, scalars: *const u64, n: usize,
                   out_jac: *mut u64, abort_cb: ecg_abort_cb, user: *mut c_void) -> c_int;
    pub fn ecg_msm_multi(ctxs: *mut *mut ecg_ctx, nctx: c_int, curve_id: c_int, bases_xy: *const u64,
                         scalars: *const u64, n: usize, out_jac: *mut u64, abort_cb: ecg_abort_cb,
                         user: *mut c_void) -> c_int;
    pub fn ecg_msm_dev(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, d_scalars: *const c_void,
                       n: usize, out_jac: *mut c_void, out_on_device: c_int, stream: *mut c_void) -> c_int;
    pub fn ecg_msm_prepare_bases(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, n: usize,
                                 d_prepared: *mut *mut c_void) -> c_int;
    pub fn ecg_msm_prepare_table(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, n: usize,
                                 window_bits: u32, d_prepared: *mut *mut c_void) -> c_int;
    pub fn ecg_msm_prepared_stride(curve_id: c_int, window_bits: u32) -> usize;
    pub fn ecg_msm_table_window(curve_id: c_int, n: usize) -> u32;
    pub fn ecg_multiple_multiexp(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, n_bases: usize,
                                 scalars: *const u64, scalars_on_device: c_int, scalars_montgomery: c_int,
                                 line_len: usize, num_chunks: usize, window_bits: u32,
                                 out_jac: *mut u64) -> c_int;

    // ---- MSM with the host-side prep on device (multiexp_cpu.rs:127-138, impls.rs:13,48-58) ----
    pub fn ecg_msm_ex(ctx: *mut ecg_ctx, curve_id: c_int, bases: *const c_void, bases_layout: c_int,
                      n_bases: usize, skip: usize, exps: *const u64, exps_montgomery: c_int, n_exps: usize,
                      density: *const u64, cache_bases: c_int, out_jac: *mut u64, abort_cb: ecg_abort_cb,
                      user: *mut c_void) -> c_int;
    pub fn ecg_base_cache_clear(ctx: *mut ecg_ctx);
    pub fn ecg_base_cache_keys(ctx: *mut ecg_ctx, out: *mut *const c_void, cap: usize) -> usize;
    pub fn ecg_msm_plan_info(curve_id: c_int, n: usize, window_bits: u32, c: *mut u32, windows: *mut u32,
                             sort_mode: *mut c_int) -> c_int;
    pub fn ecg_point_sum_dev(ctx: *mut ecg_ctx, curve_id: c_int, d_points: *const c_void, count: usize,
                             out_jac: *mut u64, stream: *mut c_void) -> c_int;
    pub fn ecg_point_sum(curve_id: c_int, points: *const u64, count: usize, out_jac: *mut u64) -> c_int;
    pub fn ecg_field_ops(ctx: *mut ecg_ctx, field_id: c_int, form: c_int, op: c_int, a: *const u64, b: *const u64,
                         e: u32, n: usize, out: *mut u64) -> c_int;
    pub fn ecg_msm_check_bases(curve_id: c_int, bases_xy: *const u64, scalars: *const u64, n: usize) -> c_int;

    // ---- multi-GPU over RCCL, one process per GPU ----
    pub fn ecg_comm_unique_id(out: *mut u8) -> c_int;
    pub fn ecg_comm_init(ctx: *mut ecg_ctx, nranks: c_int, rank: c_int, unique_id: *const u8) -> c_int;
    pub fn ecg_comm_destroy(ctx: *mut ecg_ctx);
    pub fn ecg_comm_set_timeout(ctx: *mut ecg_ctx, ms: u32) -> c_int;
    pub fn ecg_comm_info(ctx: *mut ecg_ctx, nranks: *mut c_int, rank: *mut c_int, device: *mut c_int,
                         bus_id: *mut c_char, bus_cap: usize, transport: *mut c_int) -> c_int;
    pub fn ecg_comm_last_exchange(ctx: *mut ecg_ctx, us: *mut f64) -> c_int;
    pub fn ecg_comm_init_host(ctx: *mut ecg_ctx, nranks: c_int, rank: c_int, xchg: ecg_xchg_cb,
                              user: *mut c_void) -> c_int;
    pub fn ecg_comm_allgather(ctx: *mut ecg_ctx, d_send: *const c_void, d_recv: *mut c_void, bytes: usize) -> c_int;
    pub fn ecg_comm_alltoall(ctx: *mut ecg_ctx, d_send: *const c_void, d_recv: *mut c_void,
                             bytes_per_peer: usize) -> c_int;
    pub fn ecg_msm_dist(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, d_scalars: *const c_void,
                        n_local: usize, out_jac: *mut u64) -> c_int;
    pub fn ecg_msm_dist_ex(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, d_scalars: *const c_void,
                           n_local: usize, out_jac: *mut u64, abort_cb: ecg_abort_cb, user: *mut c_void) -> c_int;
    pub fn ecg_msm_dist_grid(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, d_scalars: *const c_void,
                             n: usize, out_jac: *mut u64) -> c_int;
    pub fn ecg_msm_dist_grid_ex(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void,
                                d_scalars: *const c_void, n: usize, out_jac: *mut u64, abort_cb: ecg_abort_cb,
                                user: *mut c_void) -> c_int;
    pub fn ecg_msm_grid_part(ctx: *mut ecg_ctx, curve_id: c_int, d_bases: *const c_void, d_scalars: *const c_void,
                             n: usize, rank: c_int, nranks: c_int, out_jac: *mut u64, pieces: *mut c_int) -> c_int;
    pub fn ecg_fft_dist(ctx: *mut ecg_ctx, field_id: c_int, d_local: *mut c_void, omega: *const u64,
                        log_n: u32) -> c_int;
    pub fn ecg_fft_dist_ex(ctx: *mut ecg_ctx, field_id: c_int, d_local: *mut c_void, omega: *const u64,
                           log_n: u32, abort_cb: ecg_abort_cb, user: *mut c_void) -> c_int;
    pub fn ecg_fft_dist_stage1(ctx: *mut ecg_ctx, field_id: c_int, d_in: *const c_void, d_out: *mut c_void,
                               omega: *const u64, nranks: u32, rank: u32, log_n: u32) -> c_int;
    pub fn ecg_fft_dist_stage3(ctx: *mut ecg_ctx, d_in: *const c_void, d_out: *mut c_void, nranks: u32,
                               log_n: u32) -> c_int;

    // ---- device buffers (ag-cuda-ec/src/multiexp.rs:11-19, ag-cuda-proxy/src/params.rs:112-219) ----
    pub fn ecg_dev_alloc(ctx: *mut ecg_ctx, bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn ecg_dev_free(ctx: *mut ecg_ctx, d_ptr: *mut c_void);
    pub fn ecg_dev_upload(ctx: *mut ecg_ctx, d_dst: *mut c_void, src: *const c_void, bytes: usize) -> c_int;
    pub fn ecg_dev_download(ctx: *mut ecg_ctx, dst: *mut c_void, d_src: *const c_void, bytes: usize) -> c_int;

    // ---- benchmark helpers (no reference counterpart) ----
    pub fn ecg_gen_bases_dev(ctx: *mut ecg_ctx, curve_id: c_int, a: *const u64, b: *const u64, n: usize,
                             d_out: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn ecg_last_kernel_time(ctx: *mut ecg_ctx, name: *const c_char, ms_total: *mut f64,
                                launches: *mut c_int) -> c_int;
}
