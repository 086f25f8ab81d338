//! The workspace types ag-cuda-ec's signatures name -- `CudaWorkspace`,
//! `ActiveWorkspace`, `DeviceData`, `CudaResult` -- as an engine context and
//! engine-owned HBM buffers (ag-cuda-proxy/src/module.rs:14-63,
//! params.rs:173-219 in the reference, where they wrap a CUDA context, module
//! and stream).  The names stay so that 0g's call sites compile unchanged.

use std::os::raw::{c_int, c_void};
use std::sync::Arc;

use ag_types::{GpuCurveAffine, GpuField};
use ecgpu_sys as sys;
use rust_gpu_tools::{Device, GPUError, Program};

/// Failures of the batched entry points (rustacuda's `CudaError` in the
/// reference; the variants are the ones this engine can produce).
#[derive(Debug, Clone, PartialEq, Eq)]
pub enum CudaError {
    /// No GPU, or device 0 is not an MI355X.
    NoDevice,
    /// The engine refused an argument (its message).
    InvalidValue(String),
    /// A device allocation failed (its message).
    OutOfMemory(String),
    /// The kernel manifest asks for kernels libecgpu.so does not hold.
    NotFound(String),
    /// Any other engine failure: return code and message.
    Engine { code: i32, message: String },
}

impl std::fmt::Display for CudaError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "{self:?}")
    }
}

impl std::error::Error for CudaError {}

pub type CudaResult<T> = Result<T, CudaError>;

pub(crate) fn check(rc: c_int) -> CudaResult<()> {
    match rc {
        sys::ECG_OK => Ok(()),
        sys::ECG_ERR_NODEV => Err(CudaError::NoDevice),
        sys::ECG_ERR_INVALID => Err(CudaError::InvalidValue(sys::last_error())),
        sys::ECG_ERR_NOMEM => Err(CudaError::OutOfMemory(sys::last_error())),
        code => Err(CudaError::Engine { code, message: sys::last_error() }),
    }
}

impl From<GPUError> for CudaError {
    fn from(e: GPUError) -> Self {
        match e {
            GPUError::DeviceNotFound => CudaError::NoDevice,
            GPUError::KernelNotFound(m) => CudaError::NotFound(m),
            GPUError::Engine { code, message } => CudaError::Engine { code, message },
        }
    }
}

/// Engine curve id of the suite's `Affine`, from its moduli.
pub(crate) fn curve_of<A: GpuCurveAffine>() -> CudaResult<c_int> {
    let degree = if <A::Base as GpuField>::sub_field_name().is_some() { 2 } else { 1 };
    sys::curve_id(&sys::u64_limbs(&<A::Base as GpuField>::modulus()), degree,
                  &sys::u64_limbs(&<A::Scalar as GpuField>::modulus()))
        .map_err(CudaError::NotFound)
}

/// An engine context on device 0 (the reference's workspace takes device 0
/// too, ag-cuda-proxy/src/module.rs:24-42) that provides the kernels of the
/// crate's manifest.
pub struct CudaWorkspace {
    program: Arc<Program>,
}

impl CudaWorkspace {
    pub fn from_manifest(manifest: &str) -> CudaResult<Self> {
        let device = *Device::all().first().ok_or(CudaError::NoDevice)?;
        Ok(CudaWorkspace { program: Arc::new(Program::from_manifest(device, manifest)?) })
    }

    /// The workspace for one call; the engine serialises calls per context.
    pub fn activate<'a>(&'a self) -> CudaResult<ActiveWorkspace<'a>> {
        Ok(ActiveWorkspace(self))
    }
}

/// A workspace in use by one call.
pub struct ActiveWorkspace<'a>(&'a CudaWorkspace);

impl<'a> ActiveWorkspace<'a> {
    pub(crate) fn program(&self) -> &Arc<Program> {
        &self.0.program
    }

    pub(crate) fn ctx(&self) -> *mut sys::ecg_ctx {
        self.0.program.ctx()
    }
}

/// Bases resident in HBM, owned by the engine.  `size()` is the byte size of
/// the device buffer (prepared records: n x ecg_msm_prepared_stride, which
/// includes the window-table rows of a table upload); `len()` the bases.
pub struct DeviceData {
    program: Arc<Program>,
    ptr: *mut c_void,
    size: usize,
    len: usize,
}

unsafe impl Send for DeviceData {}
unsafe impl Sync for DeviceData {}

impl DeviceData {
    pub(crate) fn from_raw(program: Arc<Program>, ptr: *mut c_void, size: usize, len: usize) -> Self {
        DeviceData { program, ptr, size, len }
    }

    pub(crate) fn as_ptr(&self) -> *const c_void {
        self.ptr
    }

    /// Bytes of the device buffer.
    pub fn size(&self) -> usize {
        self.size
    }

    /// Elements (bases) held.
    pub fn len(&self) -> usize {
        self.len
    }

    pub fn is_empty(&self) -> bool {
        self.len == 0
    }
}

impl Drop for DeviceData {
    fn drop(&mut self) {
        unsafe { sys::ecg_dev_free(self.program.ctx(), self.ptr) }
    }
}
