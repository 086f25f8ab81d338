//! Multi-scalar multiplication on MI355X (feature `amd`): the public API of
//! ec-gpu-proxy/src/multiexp.rs (SingleMultiexpKernel 52-252, MultiexpKernel
//! 256-404) over libecgpu.so's sorted-bucket Pippenger.
//!
//! The reference converts every base on the host (`to_gpu_repr`, :152-153) and
//! copies bases and exponents in on every call (:163-164).  Here the caller's
//! arkworks `Affine { x, y, infinity }` records go to the device as they are
//! and are converted there (`ecg_msm_ex`, `ECG_BASES_ARK_AFFINE`), and
//! `MultiexpKernel::multiexp`, which receives the bases as an
//! `Arc<Vec<G>>` (immutable while shared), asks the engine to keep them
//! resident in its base cache (`cache_bases`), keyed by address: a second call
//! with the same `Arc` uploads only the exponents.  The kernel holds a clone
//! of every `Arc` the engine caches, so no other array can take a cached
//! address while its entry lives.

use std::os::raw::{c_int, c_void};
use std::sync::{Arc, RwLock};

use ag_types::{GpuCurveAffine, GpuName, GpuRepr, PrimeFieldRepr as PrimeField};
use ark_ff::Zero;
use ec_gpu_program::{EcError, EcResult};
use ecgpu_ark::{ark_layout, ArkLayout};
use ecgpu_sys as sys;
use log::{error, info, warn};
use rust_gpu_tools::{Device, Program};
use yastl::Scope;

use super::{abort_hook, check, curve_id, require, MaybeAbort};
use crate::threadpool::Worker;

/// Multiexp on one device.
pub struct SingleMultiexpKernel<'a, G>
where G: GpuCurveAffine
{
    program: Program,
    /// Terms per device pass: the engine's per-term workspace against the
    /// device memory left after the resident bases (calc_chunk_size's role,
    /// multiexp.rs:71-93).
    n: usize,
    curve: i32,
    layout: ArkLayout,
    maybe_abort: Option<&'a (dyn Fn() -> bool + Send + Sync)>,
    _phantom: std::marker::PhantomData<G::Scalar>,
}

impl<'a, G> SingleMultiexpKernel<'a, G>
where G: GpuCurveAffine + GpuName
{
    /// A kernel on `program`, whose context lives on `device`;
    /// `maybe_abort` is polled before each device pass.
    pub fn create(
        program: Program, device: &Device,
        maybe_abort: Option<&'a (dyn Fn() -> bool + Send + Sync)>,
    ) -> EcResult<Self> {
        let curve = curve_id::<G>()?;
        let mut n = 0usize;
        check(unsafe { sys::ecg_msm_chunk_size(program.ctx(), curve, &mut n) })?;
        let layout = ark_layout::<G>();
        if !layout.ark_affine {
            warn!("arkworks Affine is not laid out as {{x, y, infinity}}: bases go over in their GPU form");
        }
        info!("Multiexp on {} ({} GB, {} CUs): {} terms per pass", device.name(),
              device.memory() >> 30, device.compute_units(), n);
        Ok(SingleMultiexpKernel { program, n, curve, layout, maybe_abort, _phantom: std::marker::PhantomData })
    }

    /// sum_i exponents[i] * bases[i].  The arkworks records are read on the
    /// device (no host `to_gpu_repr` pass); exponents are canonical `BigInt`s;
    /// any length (the engine splits into passes).
    pub fn multiexp(
        &self, bases: &[G], exponents: &[<G::Scalar as PrimeField>::Repr],
    ) -> EcResult<G::Curve> {
        self.multiexp_cached(bases, exponents, false)
    }

    /// `multiexp`, with `cache` asking the engine to keep these bases resident
    /// (keyed by address and length) for later calls on the same array.
    fn multiexp_cached(
        &self, bases: &[G], exponents: &[<G::Scalar as PrimeField>::Repr], cache: bool,
    ) -> EcResult<G::Curve> {
        assert_eq!(bases.len(), exponents.len());
        require(&self.program, sys::ECG_KIND_MULTIEXP, self.curve)?;
        if !self.layout.projective_xyz {
            return Err(EcError::Simple(ecgpu_ark::NOT_XYZ));
        }
        let words = std::mem::size_of::<G::Curve>() / 8;
        let mut out = vec![0u64; words];
        let (cb, user) = abort_hook(&self.maybe_abort);
        let rc = if self.layout.ark_affine {
            unsafe {
                sys::ecg_msm_ex(self.program.ctx(), self.curve, bases.as_ptr() as *const c_void,
                                sys::ECG_BASES_ARK_AFFINE, bases.len(), 0, exponents.as_ptr() as *const u64, 0,
                                exponents.len(), std::ptr::null(), cache as c_int, out.as_mut_ptr(), cb, user)
            }
        } else {
            // the reference's own host conversion (multiexp.rs:152-153)
            let repr: Vec<_> = bases.iter().map(GpuRepr::to_gpu_repr).collect();
            unsafe {
                sys::ecg_msm(self.program.ctx(), self.curve, repr.as_ptr() as *const u64,
                             exponents.as_ptr() as *const u64, exponents.len(), out.as_mut_ptr(), cb, user)
            }
        };
        check(rc)?;
        let mut acc = G::Curve::zero();
        // layout checked by ark_layout: [X | Y | Z], every bit pattern of the
        // limbs a valid field element (the engine returns them fully reduced)
        unsafe {
            std::ptr::copy_nonoverlapping(out.as_ptr() as *const u8, &mut acc as *mut G::Curve as *mut u8,
                                          std::mem::size_of::<G::Curve>());
        }
        Ok(acc)
    }

    /// Host addresses of the base arrays this kernel's context keeps resident.
    fn cached_keys(&self) -> Vec<usize> {
        let mut keys = [std::ptr::null::<c_void>(); 8];
        let n = unsafe { sys::ecg_base_cache_keys(self.program.ctx(), keys.as_mut_ptr(), keys.len()) };
        keys[..n.min(keys.len())].iter().map(|&p| p as usize).collect()
    }
}

/// One multiexp kernel per device.
pub struct MultiexpKernel<'a, G>
where G: GpuCurveAffine
{
    kernels: Vec<SingleMultiexpKernel<'a, G>>,
    /// Base arrays the engine's caches hold on device (keyed by address):
    /// kept alive while any context caches a range of them.
    pinned: Vec<Arc<Vec<G>>>,
}

impl<'a, G> MultiexpKernel<'a, G>
where G: GpuCurveAffine + GpuName
{
    /// One kernel per (program, device) pair.
    pub fn create(
        programs: Vec<Program>, devices: &[&Device],
    ) -> EcResult<Self> {
        Self::create_optional_abort(programs, devices, None)
    }

    /// One kernel per (program, device) pair, each polling `maybe_abort`.
    pub fn create_with_abort(
        programs: Vec<Program>, devices: &[&Device],
        maybe_abort: &'a (dyn Fn() -> bool + Send + Sync),
    ) -> EcResult<Self> {
        Self::create_optional_abort(programs, devices, Some(maybe_abort))
    }

    fn create_optional_abort(
        programs: Vec<Program>, devices: &[&Device], maybe_abort: MaybeAbort<'a>,
    ) -> EcResult<Self> {
        let mut kernels = Vec::with_capacity(programs.len());
        for (program, device) in programs.into_iter().zip(devices.iter()) {
            let name = program.device_name().to_string();
            match SingleMultiexpKernel::create(program, device, maybe_abort) {
                Ok(k) => kernels.push(k),
                Err(e) => error!("Cannot initialize kernel for device '{}'! Error: {}", name, e),
            }
        }
        if kernels.is_empty() {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        info!("Multiexp: {} MI355X context(s)", kernels.len());
        Ok(MultiexpKernel { kernels, pinned: Vec::new() })
    }

    /// Device d sums the d-th of ceil(n / #devices)-term ranges, in passes of
    /// its kernel's `n` terms, on a task of `scope`; a failure is stored in
    /// `error` and every device stops before its next pass.  `results[d]`
    /// receives device d's partial sum when no device failed.
    pub fn parallel_multiexp<'s>(
        &'s mut self, scope: &Scope<'s>, bases: &'s [G],
        exps: &'s [<G::Scalar as PrimeField>::Repr],
        results: &'s mut [G::Curve], error: Arc<RwLock<EcResult<()>>>,
    ) {
        // borrowed slices of unknown lifetime: never cached
        Self::split(&self.kernels, scope, bases, exps, results, error, false)
    }

    fn split<'s>(
        kernels: &'s [SingleMultiexpKernel<'a, G>], scope: &Scope<'s>, bases: &'s [G],
        exps: &'s [<G::Scalar as PrimeField>::Repr], results: &'s mut [G::Curve],
        error: Arc<RwLock<EcResult<()>>>, cache: bool,
    ) {
        let per_device = (exps.len() + kernels.len() - 1) / kernels.len().max(1);
        if per_device == 0 {
            return;
        }
        let ranges = bases.chunks(per_device).zip(exps.chunks(per_device));
        for ((kern, (bs, es)), slot) in kernels.iter().zip(ranges).zip(results.iter_mut()) {
            let error = error.clone();
            scope.execute(move || {
                let mut partial = G::Curve::zero();
                for (b, e) in bs.chunks(kern.n).zip(es.chunks(kern.n)) {
                    if error.read().unwrap().is_err() {
                        return;
                    }
                    match kern.multiexp_cached(b, e, cache) {
                        Ok(p) => partial += p,
                        Err(err) => {
                            *error.write().unwrap() = Err(err);
                            return;
                        }
                    }
                }
                if error.read().unwrap().is_ok() {
                    *slot = partial;
                }
            });
        }
    }

    /// sum over i of exps[i] * bases_arc[skip + i] across every device; the
    /// per-device partials are added on the host (multiexp.rs:372-400).  The
    /// bases stay resident on the devices for the next call with this `Arc`.
    pub fn multiexp(
        &mut self, pool: &Worker, bases_arc: Arc<Vec<G>>,
        exps: Arc<Vec<<G::Scalar as PrimeField>::Repr>>, skip: usize,
    ) -> EcResult<G::Curve> {
        let bases = &bases_arc[skip..(skip + exps.len())];
        let exps = &exps[..];
        let mut partials = vec![G::Curve::zero(); self.kernels.len()];
        let error = Arc::new(RwLock::new(Ok(())));
        let kernels = &self.kernels;
        pool.scoped(|s| Self::split(kernels, s, bases, exps, &mut partials, error.clone(), true));
        if !self.pinned.iter().any(|a| Arc::ptr_eq(a, &bases_arc)) {
            self.pinned.push(bases_arc.clone());
        }
        self.release_uncached();
        Arc::try_unwrap(error).expect("only one ref left").into_inner().unwrap()?;
        Ok(partials.into_iter().fold(G::Curve::zero(), |acc, p| acc + p))
    }

    /// Drop the pinned arrays no context caches any more (the engine keeps
    /// at most 8 entries per context and evicts the oldest).
    fn release_uncached(&mut self) {
        let keys: Vec<usize> = self.kernels.iter().flat_map(|k| k.cached_keys()).collect();
        let size = std::mem::size_of::<G>();
        self.pinned.retain(|a| {
            let lo = a.as_ptr() as usize;
            let hi = lo + a.len() * size;
            keys.iter().any(|&k| k >= lo && k < hi)
        });
    }

    /// Kernels (devices) in use.
    pub fn num_kernels(&self) -> usize {
        self.kernels.len()
    }
}
