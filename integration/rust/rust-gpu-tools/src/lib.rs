//! The part of `rust-gpu-tools` 0.7 that the ec-gpu path touches -- `Device`,
//! `Framework`, `Program`, `GPUError` -- backed by libecgpu.so on MI355X.
//! Patched in for the crates.io package (`[patch.crates-io] rust-gpu-tools =
//! { path = ... }`) so that `use rust_gpu_tools::Device`,
//! `Device::all()` and `program.device_name()` in the reference's own crates,
//! tests and benches (ec-gpu-proxy/tests/multiexp.rs:16,43,
//! ec-gpu-proxy/src/multiexp.rs:13,109-127) keep compiling unchanged.
//!
//! There is no CUDA or OpenCL here: a `Program` is one engine context (one
//! device, one HIP stream, a grow-only device workspace) and the kernels it
//! runs are compiled into libecgpu.so ahead of time.  `program_closures!` /
//! `Program::run` have no counterpart; the ec-gpu-proxy `amd` modules call the
//! engine directly.

use std::ffi::CStr;
use std::os::raw::{c_char, c_int};
use std::sync::OnceLock;

use ecgpu_sys as sys;

/// Errors of the device layer (rust_gpu_tools::GPUError).
#[derive(Debug, Clone, PartialEq, Eq)]
pub enum GPUError {
    /// No device with that index / no GPU at all.
    DeviceNotFound,
    /// The engine refused or failed a call: its return code and message.
    Engine { code: i32, message: String },
    /// A kernel the program was asked to provide is not in libecgpu.so.
    KernelNotFound(String),
}

impl std::fmt::Display for GPUError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        match self {
            GPUError::DeviceNotFound => write!(f, "Device not found"),
            GPUError::Engine { code, message } => write!(f, "libecgpu error {code}: {message}"),
            GPUError::KernelNotFound(what) => write!(f, "Kernel not found: {what}"),
        }
    }
}

impl std::error::Error for GPUError {}

pub type GPUResult<T> = Result<T, GPUError>;

fn engine(code: c_int) -> GPUError {
    GPUError::Engine { code, message: sys::last_error() }
}

/// The compute framework of a device.  The reference selects CUDA or OpenCL
/// (ec-gpu-program/src/program.rs:64-95); this build has exactly one.
#[derive(Debug, Clone, Copy, PartialEq, Eq, Hash)]
pub enum Framework {
    /// HIP on gfx950 through libecgpu.so.
    Hip,
}

/// One MI355X, as the HIP runtime reports it.
#[derive(Debug)]
pub struct Device {
    index: c_int,
    name: String,
    memory: u64,
    compute_units: u32,
}

static DEVICES: OnceLock<Vec<Device>> = OnceLock::new();

impl Device {
    /// Every visible GPU, enumerated once per process (empty when there is
    /// none; callers map that to "No working GPUs found!").
    pub fn all() -> Vec<&'static Device> {
        DEVICES
            .get_or_init(|| {
                let n = unsafe { sys::ecg_device_count() };
                (0..n).filter_map(|i| Device::query(i).ok()).collect()
            })
            .iter()
            .collect()
    }

    fn query(index: c_int) -> GPUResult<Device> {
        let (mut mem, mut cus) = (0usize, 0 as c_int);
        let mut name = [0 as c_char; 256];
        let rc = unsafe { sys::ecg_device_info(index, &mut mem, &mut cus, name.as_mut_ptr(), name.len()) };
        if rc != sys::ECG_OK {
            return Err(engine(rc));
        }
        Ok(Device {
            index,
            name: unsafe { CStr::from_ptr(name.as_ptr()) }.to_string_lossy().into_owned(),
            memory: mem as u64,
            compute_units: cus as u32,
        })
    }

    pub fn name(&self) -> String {
        self.name.clone()
    }

    /// Device memory in bytes (288 GB of HBM3E on MI355X).
    pub fn memory(&self) -> u64 {
        self.memory
    }

    pub fn compute_units(&self) -> u32 {
        self.compute_units
    }

    /// CUDA compute capability; `None` on HIP (the reference's `work_units`
    /// falls back to its non-CUDA rule, ec-gpu-proxy/src/multiexp.rs:42-49).
    pub fn compute_capability(&self) -> Option<(u32, u32)> {
        None
    }

    pub fn framework(&self) -> Framework {
        Framework::Hip
    }

    /// HIP device ordinal.
    pub fn hip_device(&self) -> i32 {
        self.index
    }
}

/// One engine context on one device.  Every engine call takes the context's
/// lock, so a `Program` shared between threads is used by one at a time.
pub struct Program {
    ctx: *mut sys::ecg_ctx,
    device_name: String,
    /// `(kind, id)` of every kernel the manifest asked for
    kernels: Vec<(c_int, c_int)>,
}

unsafe impl Send for Program {}
unsafe impl Sync for Program {}

impl Program {
    /// A context on `device` that must provide every kernel named in
    /// `manifest` (the text `ag_build::generate` wrote): the HIP counterpart
    /// of `cuda::Program::from_bytes(device, fatbin)`.
    pub fn from_manifest(device: &Device, manifest: &str) -> GPUResult<Program> {
        let requests = sys::manifest::parse(manifest).map_err(GPUError::KernelNotFound)?;
        let kernels = sys::manifest::resolve(&requests).map_err(GPUError::KernelNotFound)?;
        let mut ctx = std::ptr::null_mut();
        let rc = unsafe { sys::ecg_ctx_create(device.index, &mut ctx) };
        if rc == sys::ECG_ERR_NODEV {
            return Err(GPUError::DeviceNotFound);
        }
        if rc != sys::ECG_OK {
            return Err(engine(rc));
        }
        Ok(Program { ctx, device_name: device.name(), kernels })
    }

    pub fn device_name(&self) -> &str {
        &self.device_name
    }

    /// Whether the manifest this program was built from asked for `(kind, id)`.
    pub fn provides(&self, kind: i32, id: i32) -> bool {
        self.kernels.contains(&(kind, id))
    }

    /// The engine context (for the crates that call libecgpu.so directly).
    pub fn ctx(&self) -> *mut sys::ecg_ctx {
        self.ctx
    }
}

impl Drop for Program {
    fn drop(&mut self) {
        unsafe { sys::ecg_ctx_destroy(self.ctx) }
    }
}
