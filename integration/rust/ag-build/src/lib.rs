//! `ag-build` for the MI355X engine: the same `SourceBuilder` chain and
//! `generate` a downstream `build.rs` already calls (ag-cuda-ec/build.rs:1-11,
//! ec-gpu-proxy/tests/multiexp.rs:34-36), with libecgpu.so behind it.
//!
//! The reference writes CUDA/OpenCL source for every requested field, curve,
//! FFT and multiexp and compiles it with nvcc (ag-build/src/source/
//! builder.rs:35-152, compile.rs:41-161).  The engine's HIP kernels for gfx950
//! are compiled into libecgpu.so ahead of time, so here a builder collects the
//! same requests -- each field named by its modulus, each curve by its
//! coordinate and scalar moduli -- and `generate` checks every one against the
//! library (a request it cannot serve fails the build, as an nvcc error would)
//! and writes them as the kernel manifest `program!` embeds.

use std::collections::BTreeSet;
use std::path::PathBuf;

use ag_types::{GpuCurveAffine, GpuField};
use ecgpu_sys::manifest::{self, Request};
use ecgpu_sys::{ECG_KIND_EC, ECG_KIND_EC_FFT, ECG_KIND_FFT, ECG_KIND_FIELD, ECG_KIND_MULTIEXP};

/// Environment variable carrying the manifest path, at compile time
/// (`cargo:rustc-env`, read by `program!`) or in the process (`load_program!`).
pub const MANIFEST_ENV: &str = "_EC_GPU_AMD_KERNEL_MANIFEST";

/// The kernels a crate needs, in the reference's builder order: fields,
/// extension fields, curves, FFTs, EC-FFTs, multiexps (builder.rs:140-151).
#[derive(Default)]
pub struct SourceBuilder {
    fields: BTreeSet<Request>,
    extension_fields: BTreeSet<Request>,
    ffts: BTreeSet<Request>,
    ec: BTreeSet<Request>,
    ec_ffts: BTreeSet<Request>,
    multiexps: BTreeSet<Request>,
    extra_sources: Vec<String>,
}

fn field_request<F: GpuField>(kind: i32) -> Request {
    let degree = if F::sub_field_name().is_some() { 2 } else { 1 };
    Request { kind, degree, modulus: ecgpu_sys::u64_limbs(&F::modulus()), scalar: None }
}

fn curve_request<C: GpuCurveAffine>(kind: i32) -> Request {
    let base = field_request::<C::Base>(kind);
    Request {
        kind,
        degree: base.degree,
        modulus: base.modulus,
        scalar: Some(ecgpu_sys::u64_limbs(&<C::Scalar as GpuField>::modulus())),
    }
}

impl SourceBuilder {
    pub fn new() -> Self {
        Self::default()
    }

    /// Request a field; an extension field brings its prime sub-field too.
    pub fn add_field<F>(mut self) -> Self
    where F: GpuField + 'static {
        let req = field_request::<F>(ECG_KIND_FIELD);
        if req.degree > 1 {
            self.fields.insert(Request { degree: 1, ..req.clone() });
            self.extension_fields.insert(req);
        } else {
            self.fields.insert(req);
        }
        self
    }

    /// Request the radix FFT over `F` (FftKernel<F>).
    pub fn add_fft<F>(self) -> Self
    where F: GpuField + 'static {
        let mut b = self.add_field::<F>();
        b.ffts.insert(field_request::<F>(ECG_KIND_FFT));
        b
    }

    /// Request the curve's group law with both of its fields.
    pub fn add_ec<C>(self) -> Self
    where C: GpuCurveAffine + 'static {
        let mut b = self.add_field::<C::Base>().add_field::<C::Scalar>();
        b.ec.insert(curve_request::<C>(ECG_KIND_EC));
        b
    }

    /// Request the FFT over the curve's points (EcFftKernel<C>).
    pub fn add_ec_fft<C>(self) -> Self
    where C: GpuCurveAffine + 'static {
        let mut b = self.add_ec::<C>();
        b.ec_ffts.insert(curve_request::<C>(ECG_KIND_EC_FFT));
        b
    }

    /// Request multiexp over the curve (MultiexpKernel<C>, multiple_multiexp).
    pub fn add_multiexp<C>(self) -> Self
    where C: GpuCurveAffine + 'static {
        let mut b = self.add_ec::<C>();
        b.multiexps.insert(curve_request::<C>(ECG_KIND_MULTIEXP));
        b
    }

    /// Extra kernel source.  Kept in the manifest as a comment; the engine
    /// does not compile source at build time, so `generate` warns that such
    /// kernels need a HIP build of their own.
    pub fn append_source(mut self, source: String) -> Self {
        self.extra_sources.push(source);
        self
    }

    /// The manifest.  The engine picks its own limb form per kernel (29-bit
    /// reduced-radix limbs on v_mad_u64_u32), so both limb-size builds name
    /// the same kernels.
    pub fn build_32_bit_limbs(&self) -> String {
        self.build()
    }

    /// See [`SourceBuilder::build_32_bit_limbs`].
    pub fn build_64_bit_limbs(&self) -> String {
        self.build()
    }

    fn build(&self) -> String {
        let all = [&self.fields, &self.extension_fields, &self.ec, &self.ffts, &self.ec_ffts, &self.multiexps];
        let mut text = manifest::render(all.iter().flat_map(|set| set.iter()));
        for (i, src) in self.extra_sources.iter().enumerate() {
            text.push_str(&format!("# appended source {i}: {} bytes (not compiled)\n", src.len()));
        }
        text
    }

    fn has_extra_sources(&self) -> bool {
        !self.extra_sources.is_empty()
    }
}

fn in_build_script() -> bool {
    std::env::var("OUT_DIR").is_ok()
}

fn working_dir() -> PathBuf {
    std::env::var("ARK_GPU_BUILD_DIR")
        .or_else(|_| std::env::var("OUT_DIR"))
        .map(PathBuf::from)
        .unwrap_or_else(|_| std::env::temp_dir())
}

/// Check every request against libecgpu.so and publish the manifest: in a
/// build script as `cargo:rustc-env=_EC_GPU_AMD_KERNEL_MANIFEST=<path>` (for
/// `program!`), otherwise in this process's environment (for `load_program!`),
/// as the reference does with its fatbin path (compile.rs:115-126).
/// Panics, failing the build, when the library lacks a requested kernel.
pub fn generate(source_builder: &SourceBuilder) {
    let text = source_builder.build_64_bit_limbs();
    let requests = manifest::parse(&text).expect("ag_build: manifest round trip");
    if let Err(e) = manifest::resolve(&requests) {
        panic!("ag_build::generate: {e}");
    }
    let path = working_dir().join("ecgpu_kernels.manifest");
    std::fs::write(&path, &text)
        .unwrap_or_else(|e| panic!("Cannot write the kernel manifest at {}: {e}", path.display()));
    if in_build_script() {
        if source_builder.has_extra_sources() {
            println!("cargo:warning=ag_build: appended kernel sources are not compiled by the MI355X engine");
        }
        println!("cargo:rustc-env={MANIFEST_ENV}={}", path.display());
        println!("cargo:rerun-if-env-changed=ECGPU_LIB_DIR");
    } else {
        std::env::set_var(MANIFEST_ENV, &path);
    }
}
