//! libecgpu.so for Rust: the raw C ABI (`ffi`, re-exported at the top level)
//! plus the few safe helpers the replacement crates share -- error text, id
//! resolution from moduli, and the kernel manifest that `ag_build::generate`
//! writes and `ec_gpu_program::program!` checks.
#![allow(non_camel_case_types, dead_code)]

mod ffi;
pub use ffi::*;

use std::ffi::CStr;
use std::fmt::Write as _;
use std::os::raw::c_int;

/// The calling thread's `ecg_last_error()` text.
pub fn last_error() -> String {
    unsafe { CStr::from_ptr(ecg_last_error()) }.to_string_lossy().into_owned()
}

/// 32-bit little-endian limbs (ag_types::GpuField::modulus) as u64 limbs.
pub fn u64_limbs(limbs32: &[u32]) -> Vec<u64> {
    limbs32
        .chunks(2)
        .map(|w| w[0] as u64 | (w.get(1).copied().unwrap_or(0) as u64) << 32)
        .collect()
}

/// Engine field id of the degree-`degree` field over `modulus` (u64 limbs).
pub fn field_id(modulus: &[u64], degree: u32) -> Result<c_int, String> {
    let id = unsafe { ecg_field_id(modulus.as_ptr(), modulus.len(), degree) };
    if id < 0 { Err(last_error()) } else { Ok(id) }
}

/// Engine curve id from its coordinate field and its scalar field.
pub fn curve_id(base: &[u64], base_degree: u32, scalar: &[u64]) -> Result<c_int, String> {
    let id = unsafe { ecg_curve_id(base.as_ptr(), base.len(), base_degree, scalar.as_ptr(), scalar.len()) };
    if id < 0 { Err(last_error()) } else { Ok(id) }
}

/// The kernel manifest: what a `SourceBuilder` asked for, one line per
/// request, `<kind> <degree> <modulus> [<scalar modulus>]` with hex moduli.
/// It is the "kernel source" of this engine: the kernels themselves are
/// compiled into libecgpu.so, so the manifest only has to name them.
pub mod manifest {
    use super::*;

    #[derive(Clone, Debug, PartialEq, Eq, PartialOrd, Ord)]
    pub struct Request {
        /// `ECG_KIND_*`
        pub kind: c_int,
        /// extension degree of the (coordinate) field
        pub degree: u32,
        /// field modulus, or the curve's coordinate-field modulus
        pub modulus: Vec<u64>,
        /// the curve's scalar modulus (curve kinds only)
        pub scalar: Option<Vec<u64>>,
    }

    const KINDS: [(&str, c_int); 5] = [
        ("field", ECG_KIND_FIELD),
        ("fft", ECG_KIND_FFT),
        ("ec", ECG_KIND_EC),
        ("ec_fft", ECG_KIND_EC_FFT),
        ("multiexp", ECG_KIND_MULTIEXP),
    ];

    fn hex(m: &[u64]) -> String {
        let mut s = String::from("0x");
        let top = m.iter().rposition(|&w| w != 0).unwrap_or(0);
        for (i, w) in m[..=top].iter().rev().enumerate() {
            if i == 0 { write!(s, "{w:x}").unwrap() } else { write!(s, "{w:016x}").unwrap() }
        }
        s
    }

    fn unhex(s: &str) -> Result<Vec<u64>, String> {
        let digits = s.strip_prefix("0x").ok_or_else(|| format!("bad modulus {s:?}"))?;
        let mut out = Vec::new();
        let mut end = digits.len();
        while end > 0 {
            let start = end.saturating_sub(16);
            out.push(u64::from_str_radix(&digits[start..end], 16).map_err(|e| format!("{s}: {e}"))?);
            end = start;
        }
        Ok(out)
    }

    /// Render requests in order, under a header line.
    pub fn render<'a>(requests: impl IntoIterator<Item = &'a Request>) -> String {
        let mut s = String::from("# libecgpu.so kernel manifest (ag_build::generate)\n");
        for r in requests {
            let kind = KINDS.iter().find(|k| k.1 == r.kind).map(|k| k.0).unwrap_or("?");
            write!(s, "{kind} {} {}", r.degree, hex(&r.modulus)).unwrap();
            if let Some(sc) = &r.scalar {
                write!(s, " {}", hex(sc)).unwrap();
            }
            s.push('\n');
        }
        s
    }

    /// Parse a rendered manifest; `#` lines and blank lines are skipped.
    pub fn parse(text: &str) -> Result<Vec<Request>, String> {
        let mut out = Vec::new();
        for line in text.lines().map(str::trim).filter(|l| !l.is_empty() && !l.starts_with('#')) {
            let f: Vec<&str> = line.split_whitespace().collect();
            let kind = KINDS.iter().find(|k| k.0 == f[0]).map(|k| k.1)
                .ok_or_else(|| format!("unknown kernel kind in manifest line {line:?}"))?;
            let curve = kind >= ECG_KIND_EC;
            if f.len() != if curve { 4 } else { 3 } {
                return Err(format!("malformed manifest line {line:?}"));
            }
            out.push(Request {
                kind,
                degree: f[1].parse().map_err(|_| format!("bad degree in {line:?}"))?,
                modulus: unhex(f[2])?,
                scalar: if curve { Some(unhex(f[3])?) } else { None },
            });
        }
        Ok(out)
    }

    /// Resolve every request against the loaded library: `(kind, id)` per
    /// request, or the first request it cannot serve, as an error text.
    pub fn resolve(requests: &[Request]) -> Result<Vec<(c_int, c_int)>, String> {
        requests
            .iter()
            .map(|r| {
                let id = match &r.scalar {
                    None => field_id(&r.modulus, r.degree)?,
                    Some(sc) => curve_id(&r.modulus, r.degree, sc)?,
                };
                if unsafe { ecg_has_kernel(r.kind, id) } == 0 {
                    return Err(format!("libecgpu.so has no {} kernel for {}", render([r]).lines().nth(1).unwrap(),
                                       name_of(r.kind, id)));
                }
                Ok((r.kind, id))
            })
            .collect()
    }

    /// `ecg_field_name` / `ecg_curve_name` of an id of `kind`.
    pub fn name_of(kind: c_int, id: c_int) -> String {
        let p = unsafe { if kind >= ECG_KIND_EC { ecg_curve_name(id) } else { ecg_field_name(id) } };
        if p.is_null() { format!("id {id}") } else { unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned() }
    }
}
