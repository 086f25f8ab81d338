//! Batched multiexp of 0g (ag-cuda-ec/src/multiexp.rs:11-81): bases uploaded
//! once, then many line x chunk MSMs sharing one exponent row.

use ag_types::{GpuRepr, PrimeFieldRepr};
use ark_std::Zero;
use ecgpu_sys as sys;

use crate::pairing_suite::{Affine, Curve, Scalar};
use crate::workspace::{check, curve_of, ActiveWorkspace, CudaError, CudaResult, DeviceData};
use crate::{GLOBAL, LOCAL};

/// Upload `bases` (their GPU form, [x, y], identity all zero) and convert them
/// once into the record layout the engine's bucket kernels gather
/// (ecg_msm_prepare_bases); the staging copy is freed before returning.
pub fn upload_multiexp_bases(
    workspace: &ActiveWorkspace, bases: &[Affine],
) -> CudaResult<DeviceData> {
    upload_prepared(workspace, bases, None)
}

/// `upload_multiexp_bases` for bases reused across many batched MSMs (0g's
/// fixed SRS / AMT bases, benches/amt.rs:18-48): besides the records, the
/// engine precomputes every base's window multiples 2^(k c) P (ecg_msm_prepare_table),
/// so each task's windows share one bucket set -- fewer mixed adds per term
/// and no per-window reduction (AMT shape: 2.65e8 instead of 1.8e8 terms/s).
/// `chunk_len` is the task length the table is sized for (exponents.len() /
/// num_chunks of the later `multiple_multiexp` calls); `window_bits = 0` lets
/// the engine pick the window for it.  Memory: ceil(256 / c) x the records.
/// Results are identical to the plain upload.
pub fn upload_multiexp_bases_table(
    workspace: &ActiveWorkspace, bases: &[Affine], chunk_len: usize, window_bits: u32,
) -> CudaResult<DeviceData> {
    let curve = curve_of::<Affine>()?;
    let c = if window_bits != 0 { window_bits } else { unsafe { sys::ecg_msm_table_window(curve, chunk_len) } };
    if c == 0 {
        return Err(CudaError::InvalidValue("no window-table form for this curve".into()));
    }
    upload_prepared(workspace, bases, Some(c))
}

fn upload_prepared(workspace: &ActiveWorkspace, bases: &[Affine], table: Option<u32>) -> CudaResult<DeviceData> {
    let curve = curve_of::<Affine>()?;
    let repr: Vec<_> = bases.iter().map(GpuRepr::to_gpu_repr).collect();
    let bytes = std::mem::size_of_val(&repr[..]);
    let ctx = workspace.ctx();
    let mut staged = std::ptr::null_mut();
    check(unsafe { sys::ecg_dev_alloc(ctx, bytes, &mut staged) })?;
    let staged = DeviceData::from_raw(workspace.program().clone(), staged, bytes, repr.len());
    check(unsafe { sys::ecg_dev_upload(ctx, staged.as_ptr() as *mut _, repr.as_ptr() as *const _, bytes) })?;
    let mut prepared = std::ptr::null_mut();
    check(unsafe {
        match table {
            None => sys::ecg_msm_prepare_bases(ctx, curve, staged.as_ptr(), repr.len(), &mut prepared),
            Some(c) => sys::ecg_msm_prepare_table(ctx, curve, staged.as_ptr(), repr.len(), c, &mut prepared),
        }
    })?;
    // the device buffer's own size: records (and table rows) per base
    let stride = unsafe { sys::ecg_msm_prepared_stride(curve, table.unwrap_or(0)) };
    Ok(DeviceData::from_raw(workspace.program().clone(), prepared, stride * repr.len(), repr.len()))
}

/// `upload_multiexp_bases_table` on this thread's workspace.
pub fn upload_multiexp_bases_table_mt(bases: &[Affine], chunk_len: usize, window_bits: u32) -> CudaResult<DeviceData> {
    LOCAL.with(|w| {
        let workspace = w.activate()?;
        upload_multiexp_bases_table(&workspace, bases, chunk_len, window_bits)
    })
}

/// `upload_multiexp_bases_table` on the global workspace.
pub fn upload_multiexp_bases_table_st(bases: &[Affine], chunk_len: usize, window_bits: u32) -> CudaResult<DeviceData> {
    let workspace = GLOBAL.activate()?;
    upload_multiexp_bases_table(&workspace, bases, chunk_len, window_bits)
}

/// `upload_multiexp_bases` on this thread's workspace.
pub fn upload_multiexp_bases_mt(bases: &[Affine]) -> CudaResult<DeviceData> {
    LOCAL.with(|w| {
        let workspace = w.activate()?;
        upload_multiexp_bases(&workspace, bases)
    })
}

/// `upload_multiexp_bases` on the global workspace.
pub fn upload_multiexp_bases_st(bases: &[Affine]) -> CudaResult<DeviceData> {
    let workspace = GLOBAL.activate()?;
    upload_multiexp_bases(&workspace, bases)
}

/// The bases form len / exponents.len() lines; each line is cut into
/// `num_chunks` chunks of exponents.len() / num_chunks terms, and output
/// [line * num_chunks + chunk] is that chunk's MSM against the same slice of
/// `exponents` (canonical `BigInt`s).  `window_size` and `neg_is_cheap` tune
/// the reference's kernel only: the engine picks its own window and always
/// uses signed digits, and the results do not depend on either.
pub fn multiple_multiexp(
    workspace: &ActiveWorkspace, bases_gpu: &DeviceData,
    exponents: &[<Scalar as PrimeFieldRepr>::Repr], num_chunks: usize,
    window_size: usize, neg_is_cheap: bool,
) -> CudaResult<Vec<Curve>> {
    let _ = (window_size, neg_is_cheap);
    let curve = curve_of::<Affine>()?;
    // the engine writes its Jacobian [X, Y, Z] results into `Curve` in place
    ecgpu_ark::require_projective_xyz::<Affine>().map_err(|m| CudaError::InvalidValue(m.into()))?;
    let num_lines = bases_gpu.len() / exponents.len();
    let mut output = vec![Curve::zero(); num_chunks * num_lines];
    check(unsafe {
        sys::ecg_multiple_multiexp(workspace.ctx(), curve, bases_gpu.as_ptr(), num_lines * exponents.len(),
                                   exponents.as_ptr() as *const u64, 0, 0, exponents.len(), num_chunks, 0,
                                   output.as_mut_ptr() as *mut u64)
    })?;
    Ok(output)
}

/// `multiple_multiexp` on this thread's workspace.
pub fn multiple_multiexp_mt(
    bases_gpu: &DeviceData, exponents: &[<Scalar as PrimeFieldRepr>::Repr], num_chunks: usize,
    window_size: usize, neg_is_cheap: bool,
) -> CudaResult<Vec<Curve>> {
    LOCAL.with(|w| {
        let workspace = w.activate()?;
        multiple_multiexp(&workspace, bases_gpu, exponents, num_chunks, window_size, neg_is_cheap)
    })
}

/// `multiple_multiexp` on the global workspace.
pub fn multiple_multiexp_st(
    bases_gpu: &DeviceData, exponents: &[<Scalar as PrimeFieldRepr>::Repr], num_chunks: usize,
    window_size: usize, neg_is_cheap: bool,
) -> CudaResult<Vec<Curve>> {
    let workspace = GLOBAL.activate()?;
    multiple_multiexp(&workspace, bases_gpu, exponents, num_chunks, window_size, neg_is_cheap)
}
