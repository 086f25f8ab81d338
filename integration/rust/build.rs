//! ec-gpu-proxy/build.rs addition for feature `amd`: link libecgpu.so from the
//! engine's build tree (ECGPU_LIB_DIR, default: the in-tree lib/ directory) and
//! embed that directory as the runtime search path.
fn main() {
    if std::env::var_os("CARGO_FEATURE_AMD").is_none() {
        return;
    }
    let dir = std::env::var("ECGPU_LIB_DIR").unwrap_or_else(|_| "../0g-ec-gpu_amd/lib".to_string());
    println!("cargo:rerun-if-env-changed=ECGPU_LIB_DIR");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=ecgpu");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
}
