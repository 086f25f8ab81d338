//! `ec-gpu-proxy` with libecgpu.so behind it (feature `amd`): the reference's
//! public kernel types with their names, signatures, error values and work
//! split, each method a call through `ffi.rs` into the HIP engine.  Replaces
//! ec-gpu-proxy/src/{fft.rs, multiexp.rs, ec_fft.rs} and ag-cuda-ec/src/{multiexp.rs,
//! ec_fft.rs} for a downstream prover; nothing else in the reference changes.
//!
//! Wiring (a maintainer's steps):
//!   * copy `ffi.rs` and this file to `ec-gpu-proxy/src/amd/{ffi,mod}.rs`;
//!   * `build.rs` (next to this file) adds the link search path of libecgpu.so;
//!   * in `ec-gpu-proxy/src/lib.rs`: `#[cfg(feature = "amd")] mod amd;
//!     #[cfg(feature = "amd")] pub use amd::{FftKernel, MultiexpKernel, EcFftKernel, ...};`
//!   * implement `FieldId` / `CurveId` for the ark types the prover uses (the
//!     ids are the `ECG_FIELD_*` / `ECG_CURVE_*` constants).
//! Element layouts are the arkworks in-memory ones (include/ecgpu.h header), so
//! slices are passed by pointer with no conversion; `G::Curve` must be the
//! 3-coordinate Jacobian `Projective` (checked in `layout_checks`).
//!
//! Not compiled in this repository (the build image has no Rust toolchain);
//! `tests/test_rust_shim.py` checks every `ffi::` call here against the header.

mod ffi;

use std::ffi::CStr;
use std::os::raw::{c_int, c_void};
use std::sync::{Arc, RwLock};

use ag_types::{GpuCurveAffine, GpuName, GpuRepr, PrimeFieldRepr};
use ark_ff::{Field, PrimeField};
use ark_std::Zero;
use ec_gpu_program::{EcError, EcResult};
use yastl::Scope;

use crate::threadpool::{Worker, THREAD_POOL};

/// Field ids of the engine (`ECG_FIELD_*`).
pub trait FieldId {
    const ID: c_int;
}
/// Curve ids of the engine (`ECG_CURVE_*`): G1 and G2 of BLS12-381 and BN254.
pub trait CurveId {
    const ID: c_int;
}

type MaybeAbort<'a> = Option<&'a (dyn Fn() -> bool + Send + Sync)>;

/// `EcError` from a return code (ec-gpu-program/src/lib.rs:10-32): 1 is
/// `Aborted`, every error code carries the thread's `ecg_last_error` text.
fn check(rc: c_int) -> EcResult<()> {
    match rc {
        ffi::ECG_OK => Ok(()),
        ffi::ECG_ABORTED => Err(EcError::Aborted),
        _ => {
            let msg = unsafe { CStr::from_ptr(ffi::ecg_last_error()) }.to_string_lossy().into_owned();
            // EcError::Simple holds a &'static str; messages are few and short-lived processes
            // rarely see more than one, so leaking them is the reference's own trade-off.
            Err(EcError::Simple(Box::leak(msg.into_boxed_str())))
        }
    }
}

/// C trampoline for `maybe_abort`: `user` points at the `&dyn Fn` the kernel holds.
unsafe extern "C" fn poll_abort(user: *mut c_void) -> c_int {
    let f = &*(user as *const &(dyn Fn() -> bool + Send + Sync));
    f() as c_int
}

fn abort_cb(maybe_abort: &MaybeAbort<'_>) -> (ffi::ecg_abort_cb, *mut c_void) {
    match maybe_abort {
        Some(f) => (Some(poll_abort), f as *const _ as *mut c_void),
        None => (None, std::ptr::null_mut()),
    }
}

// ---------------------------------------------------------------------------
// Program: `program!(device)` (ec-gpu-program/src/program.rs:11-29, 97-106)
// ---------------------------------------------------------------------------

/// One engine context: a device, its stream, a grow-only workspace and a lock
/// every call holds (so a `Program` shared across threads is used serially).
pub struct Program {
    ctx: *mut ffi::ecg_ctx,
    device: c_int,
}
unsafe impl Send for Program {}
unsafe impl Sync for Program {}

impl Program {
    /// `Device::all()` + `program!(device)` for every device: the reference's
    /// "No working GPUs found!" when there is none.
    pub fn all() -> EcResult<Vec<Program>> {
        let n = unsafe { ffi::ecg_device_count() };
        if n <= 0 {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        (0..n).map(Program::on_device).collect()
    }

    pub fn on_device(device: c_int) -> EcResult<Program> {
        let mut ctx = std::ptr::null_mut();
        check(unsafe { ffi::ecg_ctx_create(device, &mut ctx) })?;
        Ok(Program { ctx, device })
    }

    pub fn device_name(&self) -> String {
        format!("MI355X #{} ({})", self.device, unsafe {
            CStr::from_ptr(ffi::ecg_version()).to_string_lossy()
        })
    }

    /// `Device::memory()` / `compute_units()` (multiexp.rs:109-127).
    pub fn info(&self) -> EcResult<(usize, c_int)> {
        let (mut mem, mut cus) = (0usize, 0 as c_int);
        check(unsafe { ffi::ecg_ctx_info(self.ctx, &mut mem, &mut cus) })?;
        Ok((mem, cus))
    }
}

impl Drop for Program {
    fn drop(&mut self) {
        unsafe { ffi::ecg_ctx_destroy(self.ctx) }
    }
}

// ---------------------------------------------------------------------------
// FFT (ec-gpu-proxy/src/fft.rs)
// ---------------------------------------------------------------------------

/// fft.rs:19-135.
pub struct SingleFftKernel<'a, F: Field + GpuName + FieldId> {
    program: Program,
    maybe_abort: MaybeAbort<'a>,
    _phantom: std::marker::PhantomData<F>,
}

impl<'a, F: Field + GpuName + FieldId> SingleFftKernel<'a, F> {
    pub fn create(program: Program, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        Ok(SingleFftKernel { program, maybe_abort, _phantom: Default::default() })
    }

    /// In-place radix FFT of `input` (2^log_n Montgomery elements), natural
    /// order; abort polled before every pass (fft.rs:94-98).
    pub fn radix_fft(&mut self, input: &mut [F], omega: &F, log_n: u32) -> EcResult<()> {
        assert_eq!(input.len(), 1usize << log_n);
        let (cb, user) = abort_cb(&self.maybe_abort);
        check(unsafe {
            ffi::ecg_fft(self.program.ctx, F::ID, input.as_mut_ptr() as *mut u64,
                         omega as *const F as *const u64, log_n, cb, user)
        })
    }
}

/// fft.rs:139-246: every device, `radix_fft_many` split in ceil(n / #dev) chunks.
pub struct FftKernel<'a, F: Field + GpuName + FieldId> {
    kernels: Vec<SingleFftKernel<'a, F>>,
}

impl<'a, F: Field + GpuName + FieldId> FftKernel<'a, F> {
    pub fn create(programs: Vec<Program>) -> EcResult<Self> {
        Self::create_optional_abort(programs, None)
    }

    pub fn create_with_abort(programs: Vec<Program>,
                             maybe_abort: &'a (dyn Fn() -> bool + Send + Sync)) -> EcResult<Self> {
        Self::create_optional_abort(programs, Some(maybe_abort))
    }

    fn create_optional_abort(programs: Vec<Program>, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        let kernels: Vec<_> = programs.into_iter()
            .filter_map(|p| SingleFftKernel::<F>::create(p, maybe_abort).ok())
            .collect();
        if kernels.is_empty() {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        Ok(Self { kernels })
    }

    /// fft.rs:200-204: the first device.
    pub fn radix_fft(&mut self, input: &mut [F], omega: &F, log_n: u32) -> EcResult<()> {
        self.kernels[0].radix_fft(input, omega, log_n)
    }

    /// fft.rs:211-246.  The engine runs the per-device threads itself
    /// (ecg_fft_many: ceil(n / #dev) transforms per context, first error wins).
    pub fn radix_fft_many(&mut self, inputs: &mut [&mut [F]], omegas: &[F], log_ns: &[u32]) -> EcResult<()> {
        assert!(inputs.len() == omegas.len() && inputs.len() == log_ns.len());
        let mut ctxs: Vec<_> = self.kernels.iter().map(|k| k.program.ctx).collect();
        let mut ptrs: Vec<*mut u64> = inputs.iter_mut().map(|s| s.as_mut_ptr() as *mut u64).collect();
        let (cb, user) = abort_cb(&self.kernels[0].maybe_abort);
        check(unsafe {
            ffi::ecg_fft_many(ctxs.as_mut_ptr(), ctxs.len() as c_int, F::ID, ptrs.as_mut_ptr(),
                              omegas.as_ptr() as *const u64, log_ns.as_ptr(), ptrs.len(), cb, user)
        })
    }
}

// ---------------------------------------------------------------------------
// Multiexp (ec-gpu-proxy/src/multiexp.rs)
// ---------------------------------------------------------------------------

/// multiexp.rs:52-252.  `n` is the terms per device pass the engine derives
/// from device memory (`calc_chunk_size`, multiexp.rs:71-93).
pub struct SingleMultiexpKernel<'a, G: GpuCurveAffine + GpuName + CurveId> {
    program: Program,
    pub n: usize,
    maybe_abort: MaybeAbort<'a>,
    _phantom: std::marker::PhantomData<G>,
}

impl<'a, G: GpuCurveAffine + GpuName + CurveId> SingleMultiexpKernel<'a, G> {
    pub fn create(program: Program, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        let mut n = 0usize;
        check(unsafe { ffi::ecg_msm_chunk_size(program.ctx, G::ID, &mut n) })?;
        Ok(SingleMultiexpKernel { program, n, maybe_abort, _phantom: Default::default() })
    }

    /// multiexp.rs:135-236: Σ exponents[i]·bases[i].  Bases in the GPU
    /// representation (GpuRepr::to_gpu_repr, as multiexp.rs:152 builds them),
    /// exponents canonical `BigInt<4>`; abort polled before every device pass.
    pub fn multiexp(&self, bases: &[G], exponents: &[<G::Scalar as PrimeField>::Repr]) -> EcResult<G::Curve> {
        assert_eq!(bases.len(), exponents.len());
        let repr: Vec<_> = bases.iter().map(GpuRepr::to_gpu_repr).collect();
        let mut out = G::Curve::zero();
        let (cb, user) = abort_cb(&self.maybe_abort);
        check(unsafe {
            ffi::ecg_msm(self.program.ctx, G::ID, repr.as_ptr() as *const u64,
                         exponents.as_ptr() as *const u64, exponents.len(),
                         &mut out as *mut G::Curve as *mut u64, cb, user)
        })?;
        Ok(out)
    }
}

/// multiexp.rs:256-404.
pub struct MultiexpKernel<'a, G: GpuCurveAffine + GpuName + CurveId> {
    kernels: Vec<SingleMultiexpKernel<'a, G>>,
}

impl<'a, G: GpuCurveAffine + GpuName + CurveId> MultiexpKernel<'a, G> {
    pub fn create(programs: Vec<Program>) -> EcResult<Self> {
        Self::create_optional_abort(programs, None)
    }

    pub fn create_with_abort(programs: Vec<Program>,
                             maybe_abort: &'a (dyn Fn() -> bool + Send + Sync)) -> EcResult<Self> {
        Self::create_optional_abort(programs, Some(maybe_abort))
    }

    fn create_optional_abort(programs: Vec<Program>, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        let kernels: Vec<_> = programs.into_iter()
            .filter_map(|p| SingleMultiexpKernel::<G>::create(p, maybe_abort).ok())
            .collect();
        if kernels.is_empty() {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        Ok(MultiexpKernel { kernels })
    }

    /// multiexp.rs:324-367: contiguous ceil(n / #dev) ranges, one scope task
    /// per device, each range in passes of its kernel's `n` terms, the first
    /// error stops the others at their next pass; `results[d]` gets device d's
    /// partial sum.
    pub fn parallel_multiexp<'s>(&'s mut self, scope: &Scope<'s>, bases: &'s [G],
                                 exps: &'s [<G::Scalar as PrimeField>::Repr], results: &'s mut [G::Curve],
                                 error: Arc<RwLock<EcResult<()>>>) {
        let num_devices = self.kernels.len();
        let chunk_size = ((exps.len() as f64) / (num_devices as f64)).ceil() as usize;
        for (((bases, exps), kern), result) in bases.chunks(chunk_size)
            .zip(exps.chunks(chunk_size))
            .zip(self.kernels.iter_mut())
            .zip(results.iter_mut())
        {
            let error = error.clone();
            scope.execute(move || {
                let mut acc = G::Curve::zero();
                for (bases, exps) in bases.chunks(kern.n).zip(exps.chunks(kern.n)) {
                    if error.read().unwrap().is_err() {
                        break;
                    }
                    match kern.multiexp(bases, exps) {
                        Ok(r) => acc += r,
                        Err(e) => {
                            *error.write().unwrap() = Err(e);
                            break;
                        }
                    }
                }
                if error.read().unwrap().is_ok() {
                    *result = acc;
                }
            });
        }
    }

    /// multiexp.rs:372-400: `bases[skip..skip + exps.len()]`, partials folded on
    /// the host.
    pub fn multiexp(&mut self, pool: &Worker, bases_arc: Arc<Vec<G>>,
                    exps: Arc<Vec<<G::Scalar as PrimeField>::Repr>>, skip: usize) -> EcResult<G::Curve> {
        if bases_arc.len() < skip + exps.len() {
            return Err(EcError::Simple("Expected more bases from source."));
        }
        let bases = &bases_arc[skip..(skip + exps.len())];
        let exps = &exps[..];
        let mut results = vec![G::Curve::zero(); self.kernels.len()];
        let error = Arc::new(RwLock::new(Ok(())));
        pool.scoped(|s| {
            self.parallel_multiexp(s, bases, exps, &mut results, error.clone());
        });
        Arc::try_unwrap(error).expect("only one ref left").into_inner().unwrap()?;
        let mut acc = G::Curve::zero();
        for r in results {
            acc += r;
        }
        Ok(acc)
    }

    pub fn num_kernels(&self) -> usize {
        self.kernels.len()
    }
}

// ---------------------------------------------------------------------------
// EC-FFT (ec-gpu-proxy/src/ec_fft.rs)
// ---------------------------------------------------------------------------

/// ec_fft.rs:18-160: in-place DFT over G1/G2 points (`G::Curve`, Jacobian).
pub struct SingleEcFftKernel<'a, G: GpuCurveAffine + CurveId> {
    program: Program,
    maybe_abort: MaybeAbort<'a>,
    _phantom: std::marker::PhantomData<G>,
}

impl<'a, G: GpuCurveAffine + CurveId> SingleEcFftKernel<'a, G> {
    pub fn create(program: Program, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        Ok(SingleEcFftKernel { program, maybe_abort, _phantom: Default::default() })
    }

    pub fn radix_ec_fft(&mut self, input: &mut [G::Curve], omega: &G::Scalar, log_n: u32) -> EcResult<()> {
        assert_eq!(input.len(), 1usize << log_n);
        let (cb, user) = abort_cb(&self.maybe_abort);
        check(unsafe {
            ffi::ecg_ec_fft(self.program.ctx, G::ID, input.as_mut_ptr() as *mut u64,
                            omega as *const G::Scalar as *const u64, log_n, cb, user)
        })
    }
}

/// ec_fft.rs:164-280.
pub struct EcFftKernel<'a, G: GpuCurveAffine + CurveId> {
    kernels: Vec<SingleEcFftKernel<'a, G>>,
}

impl<'a, G: GpuCurveAffine + CurveId> EcFftKernel<'a, G> {
    pub fn create(programs: Vec<Program>) -> EcResult<Self> {
        Self::create_optional_abort(programs, None)
    }

    pub fn create_with_abort(programs: Vec<Program>,
                             maybe_abort: &'a (dyn Fn() -> bool + Send + Sync)) -> EcResult<Self> {
        Self::create_optional_abort(programs, Some(maybe_abort))
    }

    fn create_optional_abort(programs: Vec<Program>, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        let kernels: Vec<_> = programs.into_iter()
            .filter_map(|p| SingleEcFftKernel::<G>::create(p, maybe_abort).ok())
            .collect();
        if kernels.is_empty() {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        Ok(Self { kernels })
    }

    pub fn radix_ec_fft(&mut self, input: &mut [G::Curve], omega: &G::Scalar, log_n: u32) -> EcResult<()> {
        self.kernels[0].radix_ec_fft(input, omega, log_n)
    }

    pub fn radix_ec_fft_many(&mut self, inputs: &mut [&mut [G::Curve]], omegas: &[G::Scalar],
                             log_ns: &[u32]) -> EcResult<()> {
        assert!(inputs.len() == omegas.len() && inputs.len() == log_ns.len());
        let mut ctxs: Vec<_> = self.kernels.iter().map(|k| k.program.ctx).collect();
        let mut ptrs: Vec<*mut u64> = inputs.iter_mut().map(|s| s.as_mut_ptr() as *mut u64).collect();
        let (cb, user) = abort_cb(&self.kernels[0].maybe_abort);
        check(unsafe {
            ffi::ecg_ec_fft_many(ctxs.as_mut_ptr(), ctxs.len() as c_int, G::ID, ptrs.as_mut_ptr(),
                                 omegas.as_ptr() as *const u64, log_ns.as_ptr(), ptrs.len(), cb, user)
        })
    }
}

// ---------------------------------------------------------------------------
// ag-cuda-ec entry points (ag-cuda-ec/src/{multiexp.rs, ec_fft.rs}); the
// `#[auto_workspace]` workspace becomes a `Program`, `DeviceData` a library
// buffer in HBM.
// ---------------------------------------------------------------------------

/// A device buffer owned by the engine (ag-cuda-proxy's `DeviceData`).
pub struct DeviceData<'p> {
    program: &'p Program,
    ptr: *mut c_void,
    /// elements (bases) held
    pub n: usize,
}

impl Drop for DeviceData<'_> {
    fn drop(&mut self) {
        unsafe { ffi::ecg_dev_free(self.program.ctx, self.ptr) }
    }
}

fn upload_bases<'p, A: GpuRepr + CurveId>(ws: &'p Program, bases: &[A]) -> EcResult<DeviceData<'p>> {
    let repr: Vec<_> = bases.iter().map(GpuRepr::to_gpu_repr).collect();
    let bytes = std::mem::size_of_val(&repr[..]);
    let mut raw = std::ptr::null_mut();
    check(unsafe { ffi::ecg_dev_alloc(ws.ctx, bytes, &mut raw) })?;
    let staged = DeviceData { program: ws, ptr: raw, n: repr.len() }; // freed on return
    check(unsafe { ffi::ecg_dev_upload(ws.ctx, raw, repr.as_ptr() as *const c_void, bytes) })?;
    Ok(staged)
}

/// ag-cuda-ec/src/multiexp.rs:11-19: upload once, converted once into the
/// bucket kernels' record layout (ecg_msm_prepare_bases).
pub fn upload_multiexp_bases<'p, A: GpuRepr + CurveId>(ws: &'p Program, bases: &[A]) -> EcResult<DeviceData<'p>> {
    let staged = upload_bases(ws, bases)?;
    let mut p = std::ptr::null_mut();
    check(unsafe { ffi::ecg_msm_prepare_bases(ws.ctx, A::ID, staged.ptr, staged.n, &mut p) })?;
    Ok(DeviceData { program: ws, ptr: p, n: staged.n })
}

/// Optional (no reference counterpart): fixed bases prepared as a window
/// table (ecg_msm_prepare_table, W = ceil(256 / c) times the memory); every
/// MSM over the buffer feeds one bucket set per task.  For multiple_multiexp
/// pass the chunk length as `n_hint`.
pub fn upload_multiexp_table<'p, A: GpuRepr + CurveId>(ws: &'p Program, bases: &[A], n_hint: usize)
                                                      -> EcResult<DeviceData<'p>> {
    let staged = upload_bases(ws, bases)?;
    let c = unsafe { ffi::ecg_msm_table_window(A::ID, n_hint) };
    let mut p = std::ptr::null_mut();
    check(unsafe { ffi::ecg_msm_prepare_table(ws.ctx, A::ID, staged.ptr, staged.n, c, &mut p) })?;
    Ok(DeviceData { program: ws, ptr: p, n: staged.n })
}

/// ag-cuda-ec/src/multiexp.rs:21-81: lines × chunks MSMs over the uploaded
/// bases sharing one exponent row; `window_size` / `neg_is_cheap` tune only
/// the reference's kernel (the engine picks its window, results identical).
pub fn multiple_multiexp<A: GpuCurveAffine + CurveId>(ws: &Program, bases_gpu: &DeviceData<'_>,
                                                      exponents: &[<A::Scalar as PrimeFieldRepr>::Repr],
                                                      num_chunks: usize, _window_size: usize,
                                                      _neg_is_cheap: bool) -> EcResult<Vec<A::Curve>> {
    let lines = bases_gpu.n / exponents.len();
    let mut out = vec![A::Curve::zero(); lines * num_chunks];
    check(unsafe {
        ffi::ecg_multiple_multiexp(ws.ctx, A::ID, bases_gpu.ptr, bases_gpu.n,
                                   exponents.as_ptr() as *const u64, 0, 0, exponents.len(), num_chunks, 0,
                                   out.as_mut_ptr() as *mut u64)
    })?;
    Ok(out)
}

/// ag-cuda-ec/src/ec_fft.rs:12-93: `omegas[0]` is the transform's root of unity.
pub fn radix_ec_fft<A: GpuCurveAffine + CurveId>(ws: &Program, input: &mut Vec<A::Curve>,
                                                 omegas: &[A::Scalar]) -> EcResult<()> {
    let n = input.len();
    let log_n = n.ilog2();
    assert_eq!(n, 1 << log_n);
    check(unsafe {
        ffi::ecg_ec_fft(ws.ctx, A::ID, input.as_mut_ptr() as *mut u64, omegas.as_ptr() as *const u64, log_n,
                        None, std::ptr::null_mut())
    })
}

#[cfg(test)]
mod layout_checks {
    /// The engine writes 3 coordinates of the base field per result point.
    #[test]
    fn projective_is_three_coordinates() {
        assert_eq!(std::mem::size_of::<ark_bls12_381::G1Projective>(), 3 * 48);
        assert_eq!(std::mem::size_of::<ark_bn254::G1Projective>(), 3 * 32);
        assert_eq!(std::mem::size_of::<ark_bls12_381::G2Projective>(), 3 * 96);
        assert_eq!(std::mem::size_of::<ark_bn254::G2Projective>(), 3 * 64);
        assert_eq!(std::mem::size_of::<ark_bls12_381::Fr>(), 32);
    }
}
