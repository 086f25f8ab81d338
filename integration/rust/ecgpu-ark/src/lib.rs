//! How libecgpu.so may touch arkworks points in place.
//!
//! arkworks' short-Weierstrass `Affine { x, y, infinity: bool }` and
//! `Projective { x, y, z }` carry no `repr(C)`, so every drop-in that hands
//! `G` or `G::Curve` memory to the engine probes their field order once on the
//! curve's generator instead of assuming it (the reference reads `G::Curve`
//! straight out of a device buffer, ec-gpu-proxy/src/multiexp.rs:209-211,
//! ec_fft.rs:136-139; ag-cuda-ec/src/multiexp.rs:70-78):
//!   * `ark_affine`: x at offset 0, y right after it, the `infinity` flag in
//!     the byte after y, record size 2 coordinates + 8 -- the layout
//!     `ECG_BASES_ARK_AFFINE` reads on the device;
//!   * `projective_xyz`: `Projective::from(generator)` is the bytes of
//!     [x | y | one], i.e. the engine's Jacobian [X, Y, Z] points can be read
//!     from and written into `G::Curve`.
//! A shim that writes `G::Curve` refuses the call when `projective_xyz` is
//! false (tests/test_rust_shim.py checks that every such shim calls
//! `require_projective_xyz`).

use ark_ec::AffineRepr;
use ark_ff::One;

#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct ArkLayout {
    pub ark_affine: bool,
    pub projective_xyz: bool,
}

fn bytes_of<T>(v: &T) -> &[u8] {
    // only called on field elements and projective points: no padding bytes
    unsafe { std::slice::from_raw_parts(v as *const T as *const u8, std::mem::size_of::<T>()) }
}

/// Probe `A` and `A::Group` on the generator (cheap: one conversion).
pub fn ark_layout<A: AffineRepr>() -> ArkLayout {
    let lq = std::mem::size_of::<A::BaseField>();
    let g = A::generator();
    let (gx, gy) = match g.xy() {
        Some(xy) => xy,
        None => return ArkLayout { ark_affine: false, projective_xyz: false },
    };
    let at = |p: &A, f: &A::BaseField| f as *const _ as usize - p as *const A as usize;
    // the flag byte: the identity has it set, the generator clear (read only
    // once x and y are known to fill the first 2 lq bytes)
    let flag = |p: &A| unsafe { std::ptr::read((p as *const A as *const u8).add(2 * lq)) };
    let ark_affine = std::mem::size_of::<A>() == 2 * lq + 8
        && at(&g, gx) == 0
        && at(&g, gy) == lq
        && flag(&g) == 0
        && flag(&A::zero()) == 1;
    let p: A::Group = g.into_group();
    let one = <A::BaseField as One>::one();
    let pb = bytes_of(&p);
    let projective_xyz = pb.len() == 3 * lq
        && &pb[..lq] == bytes_of(gx)
        && &pb[lq..2 * lq] == bytes_of(gy)
        && &pb[2 * lq..] == bytes_of(&one);
    ArkLayout { ark_affine, projective_xyz }
}

/// The message every shim returns when `G::Curve` cannot be written in place.
pub const NOT_XYZ: &str = "arkworks Projective is not laid out as [x, y, z]; \
                           the engine's points cannot be read from or written into G::Curve";

/// `Err(NOT_XYZ)` unless the engine may write `A::Group` in place.
pub fn require_projective_xyz<A: AffineRepr>() -> Result<ArkLayout, &'static str> {
    let l = ark_layout::<A>();
    if l.projective_xyz { Ok(l) } else { Err(NOT_XYZ) }
}
