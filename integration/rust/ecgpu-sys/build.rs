//! Link libecgpu.so from the engine's build tree (ECGPU_LIB_DIR, default: the
//! in-tree 0g-ec-gpu_amd/lib directory) and embed that directory as the
//! runtime search path, so binaries and build scripts that use the engine
//! (ag_build::generate checks its manifest against the library) find it.
fn main() {
    let default = concat!(env!("CARGO_MANIFEST_DIR"), "/../../../0g-ec-gpu_amd/lib");
    let dir = std::env::var("ECGPU_LIB_DIR").unwrap_or_else(|_| default.to_string());
    println!("cargo:rerun-if-env-changed=ECGPU_LIB_DIR");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=ecgpu");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    // exported to dependents' build scripts as DEP_ECGPU_LIB_DIR
    println!("cargo:lib_dir={dir}");
}
