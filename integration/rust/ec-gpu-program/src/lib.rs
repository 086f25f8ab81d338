//! `ec-gpu-program` for the MI355X engine: the error type every kernel
//! returns, `program!` / `load_program!`, and the framework check, with
//! libecgpu.so in place of CUDA fatbins and OpenCL sources.
//!
//! The reference (ec-gpu-program/src/{lib.rs:9-32, program.rs:11-118})
//! embeds the kernel binary `ag_build::generate` compiled for the crate and
//! loads it per device.  Here the kernels are already in libecgpu.so;
//! `generate` records which of them the crate asked for (the manifest at
//! `_EC_GPU_AMD_KERNEL_MANIFEST`), and `program!` opens an engine context on
//! the device after checking that the library provides every one of them.

pub use rust_gpu_tools::{Device, Framework, Program};

/// Error values of every ec-gpu call, same variants and texts as the
/// reference's (ec-gpu-program/src/lib.rs:10-29).
#[derive(thiserror::Error, Debug)]
pub enum EcError {
    /// A described failure, e.g. "No working GPUs found!".
    #[error("EcError: {0}")]
    Simple(&'static str),

    /// `maybe_abort` returned true at a poll point; the device is left usable.
    #[error("GPU call was aborted!")]
    Aborted,

    /// A device-layer failure (libecgpu.so's code and message).
    #[error("GPU tools error: {0}")]
    GpuTools(#[from] rust_gpu_tools::GPUError),

    #[error("Encountered an I/O error: {0}")]
    Io(#[from] std::io::Error),
}

/// Result of every ec-gpu call.
pub type EcResult<T> = std::result::Result<T, EcError>;

/// Which framework runs `device`.  `EC_GPU_FRAMEWORK` may name "hip" (or be
/// unset); asking for "cuda" or "opencl" is refused with the reference's
/// wording, since this build has neither (program.rs:64-95).
pub fn check_framework(device: &Device) -> EcResult<Framework> {
    match std::env::var("EC_GPU_FRAMEWORK").as_deref() {
        Ok("cuda") => Err(EcError::Simple(
            "CUDA framework is not supported, please compile with the `cuda` feature enabled.",
        )),
        Ok("opencl") => Err(EcError::Simple(
            "OpenCL framework is not supported, please compile with the `opencl` feature enabled.",
        )),
        _ => Ok(device.framework()),
    }
}

/// The HIP counterpart of the reference's `build_cuda_program(device, fatbin)`
/// (program.rs:97-106): an engine context on `device` that provides every
/// kernel the manifest names.
pub fn build_hip_program(device: &Device, manifest: &str) -> EcResult<Program> {
    Ok(Program::from_manifest(device, manifest)?)
}

/// A [`Program`] for a device, from the manifest `ag_build::generate` wrote in
/// the calling crate's `build.rs` (embedded at compile time).
#[macro_export]
macro_rules! program {
    ($device:ident) => {{
        use ec_gpu_program::*;

        match check_framework($device) {
            Ok(Framework::Hip) => {
                build_hip_program($device, include_str!(env!("_EC_GPU_AMD_KERNEL_MANIFEST")))
            }
            Err(e) => Err(e),
        }
    }};
}

/// Like [`program!`] but reads the manifest at run time from the path in
/// `_EC_GPU_AMD_KERNEL_MANIFEST` (the reference's test helper, program.rs:31-60).
#[cfg(feature = "test-tools")]
#[macro_export]
macro_rules! load_program {
    ($device:ident) => {{
        use ec_gpu_program::*;

        match check_framework($device) {
            Ok(Framework::Hip) => {
                let path = std::env::var("_EC_GPU_AMD_KERNEL_MANIFEST").unwrap();
                match std::fs::read_to_string(&path) {
                    Ok(manifest) => build_hip_program($device, &manifest),
                    Err(e) => Err(EcError::Io(e)),
                }
            }
            Err(e) => Err(e),
        }
    }};
}
