//! EC-FFT of 0g (ag-cuda-ec/src/ec_fft.rs:12-99): one transform of the
//! suite's G1 points, `omegas[0]` its root of unity.

use ecgpu_sys as sys;

use crate::pairing_suite::{Affine, Curve, Scalar};
use crate::workspace::{check, curve_of, ActiveWorkspace, CudaError, CudaResult};
use crate::{GLOBAL, LOCAL};

/// `input` (2^k projective points) is replaced by its DFT at `omegas[0]`
/// (P_j = sum_i omega^(ij) P_i), natural order, written back normalised.
pub fn radix_ec_fft(
    workspace: &ActiveWorkspace, input: &mut Vec<Curve>, omegas: &[Scalar],
) -> CudaResult<()> {
    let n = input.len();
    let log_n = n.ilog2();
    assert_eq!(n, 1 << log_n);
    let curve = curve_of::<Affine>()?;
    // the engine reads and writes `Curve` as [X, Y, Z] in place
    ecgpu_ark::require_projective_xyz::<Affine>().map_err(|m| CudaError::InvalidValue(m.into()))?;
    check(unsafe {
        sys::ecg_ec_fft(workspace.ctx(), curve, input.as_mut_ptr() as *mut u64,
                        omegas.as_ptr() as *const u64, log_n, None, std::ptr::null_mut())
    })
}

/// `radix_ec_fft` on this thread's workspace.
pub fn radix_ec_fft_mt(input: &mut Vec<Curve>, omegas: &[Scalar]) -> CudaResult<()> {
    LOCAL.with(|w| {
        let workspace = w.activate()?;
        radix_ec_fft(&workspace, input, omegas)
    })
}

/// `radix_ec_fft` on the global workspace.
pub fn radix_ec_fft_st(input: &mut Vec<Curve>, omegas: &[Scalar]) -> CudaResult<()> {
    let workspace = GLOBAL.activate()?;
    radix_ec_fft(&workspace, input, omegas)
}
