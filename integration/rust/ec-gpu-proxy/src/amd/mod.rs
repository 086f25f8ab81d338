//! The GPU half of ec-gpu-proxy (feature `amd`) over libecgpu.so: `fft`,
//! `multiexp` and `ec_fft` keep the reference's public types, signatures,
//! error values and device split (ec-gpu-proxy/src/{fft,multiexp,ec_fft}.rs);
//! their bodies call the HIP engine.  Wiring, in ec-gpu-proxy/src/lib.rs
//!:
//!
//! ```ignore
//! #[cfg(feature = "amd")] mod amd;
//! #[cfg(feature = "amd")] pub use amd::{ec_fft, fft, multiexp};
//! ```
//!
//! Generic parameters keep the reference's bounds (`F: Field + GpuName`,
//! `G: GpuCurveAffine + GpuName`): the engine id of a field or curve is looked
//! up from its moduli at run time (`ecg_field_id` / `ecg_curve_id`), so no
//! extra trait is needed at any call site.

pub mod ec_fft;
pub mod fft;
pub mod multiexp;

use std::os::raw::{c_int, c_void};

use ag_types::{GpuCurveAffine, GpuField};
use ark_ff::Field;
use ec_gpu_program::{EcError, EcResult};
use ecgpu_sys as sys;
use rust_gpu_tools::{GPUError, Program};

/// `maybe_abort` as every kernel stores it.
pub(crate) type MaybeAbort<'a> = Option<&'a (dyn Fn() -> bool + Send + Sync)>;

/// Engine return code -> the reference's error values: 1 is
/// `EcError::Aborted`, any failure `EcError::GpuTools` with the engine's text.
pub(crate) fn check(rc: c_int) -> EcResult<()> {
    match rc {
        sys::ECG_OK => Ok(()),
        sys::ECG_ABORTED => Err(EcError::Aborted),
        code => Err(EcError::GpuTools(GPUError::Engine { code, message: sys::last_error() })),
    }
}

fn not_found(message: String) -> EcError {
    EcError::GpuTools(GPUError::KernelNotFound(message))
}

/// Engine field id of `F` (a prime field), from `Field::characteristic`.
pub(crate) fn field_id<F: Field>() -> EcResult<c_int> {
    sys::field_id(F::characteristic(), F::extension_degree() as u32).map_err(not_found)
}

/// Engine curve id of `G`, from its coordinate and scalar moduli.
pub(crate) fn curve_id<G: GpuCurveAffine>() -> EcResult<c_int> {
    let degree = if <G::Base as GpuField>::sub_field_name().is_some() { 2 } else { 1 };
    sys::curve_id(&sys::u64_limbs(&<G::Base as GpuField>::modulus()), degree,
                  &sys::u64_limbs(&<G::Scalar as GpuField>::modulus()))
        .map_err(not_found)
}

/// The engine runs only the kernels the program's manifest asked for, as the
/// reference runs only the kernels its generated source holds.
pub(crate) fn require(program: &Program, kind: c_int, id: c_int) -> EcResult<()> {
    if program.provides(kind, id) {
        Ok(())
    } else {
        Err(not_found(format!("{} kernel for {} (add it to the SourceBuilder in build.rs)",
                              ["field", "fft", "ec", "ec_fft", "multiexp"][kind as usize],
                              sys::manifest::name_of(kind, id))))
    }
}

/// C trampoline for `maybe_abort`: `user` points at the `&dyn Fn` a kernel holds.
unsafe extern "C" fn poll_abort(user: *mut c_void) -> c_int {
    let f = &*(user as *const &(dyn Fn() -> bool + Send + Sync));
    f() as c_int
}

/// `(callback, user)` for the engine's poll points (between FFT passes and
/// MSM device passes, fft.rs:94-98, multiexp.rs:140-144).
pub(crate) fn abort_hook(maybe_abort: &MaybeAbort<'_>) -> (sys::ecg_abort_cb, *mut c_void) {
    match maybe_abort {
        Some(f) => (Some(poll_abort), f as *const _ as *mut c_void),
        None => (None, std::ptr::null_mut()),
    }
}

#[cfg(test)]
mod layout_checks {
    /// The engine reads and writes the arkworks layouts in place: Fr as four
    /// Montgomery u64 limbs, `Projective` as X, Y, Z of the coordinate field.
    #[test]
    fn element_layouts() {
        assert_eq!(std::mem::size_of::<ark_bls12_381::Fr>(), 32);
        assert_eq!(std::mem::size_of::<ark_bn254::Fr>(), 32);
        assert_eq!(std::mem::size_of::<ark_bls12_381::G1Projective>(), 3 * 48);
        assert_eq!(std::mem::size_of::<ark_bn254::G1Projective>(), 3 * 32);
        assert_eq!(std::mem::size_of::<ark_bls12_381::G2Projective>(), 3 * 96);
        assert_eq!(std::mem::size_of::<ark_bn254::G2Projective>(), 3 * 64);
    }
}
