//! ag-cuda-ec on MI355X: 0g's batched multiexp and EC-FFT entry points
//! (ag-cuda-ec/src/{multiexp.rs, ec_fft.rs}) over libecgpu.so, with the
//! `_st` / `_mt` variants that `#[auto_workspace]` generates in the reference
//! (ag-cuda-workspace-macro/src/lib.rs:21-51) and the global / thread-local
//! workspaces of `construct_workspace!` (lib.rs:58-78) written out.
//!
//! `pairing_suite.rs` and `test_tools.rs` are the reference's own files,
//! unchanged; the crate's `build.rs` is unchanged too -- its `ag_build::
//! generate` call now writes the kernel manifest the workspaces load.

pub mod ec_fft;
pub mod multiexp;
pub mod pairing_suite;
pub mod test_tools;
mod workspace;

pub use workspace::{ActiveWorkspace, CudaError, CudaResult, CudaWorkspace, DeviceData};

/// The manifest `ag_build::generate` wrote for this crate (build.rs).
const MANIFEST: &str = include_str!(env!("_EC_GPU_AMD_KERNEL_MANIFEST"));

fn new_workspace() -> CudaWorkspace {
    CudaWorkspace::from_manifest(MANIFEST).unwrap()
}

/// The process-wide workspace the `_st` functions use.
static GLOBAL: once_cell::sync::Lazy<CudaWorkspace> = once_cell::sync::Lazy::new(new_workspace);

std::thread_local! {
    /// One workspace per thread for the `_mt` functions.
    static LOCAL: once_cell::unsync::Lazy<CudaWorkspace> = once_cell::unsync::Lazy::new(new_workspace);
}

/// Open the global workspace now rather than at the first `_st` call.
pub fn init_global_workspace() {
    once_cell::sync::Lazy::force(&GLOBAL);
}

/// Open this thread's workspace now rather than at its first `_mt` call.
pub fn init_local_workspace() {
    LOCAL.with(|w| {
        once_cell::unsync::Lazy::force(w);
    });
}
