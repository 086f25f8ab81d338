//! Multi-scalar multiplication on MI355X (feature `amd`): the public API of
//! ec-gpu-proxy/src/multiexp.rs (SingleMultiexpKernel 52-252, MultiexpKernel
//! 256-404) over libecgpu.so's sorted-bucket Pippenger (ecg_msm).

use std::sync::{Arc, RwLock};

use ag_types::{GpuCurveAffine, GpuName, GpuRepr, PrimeFieldRepr as PrimeField};
use ark_ff::Zero;
use ec_gpu_program::{EcError, EcResult};
use ecgpu_sys as sys;
use log::{error, info};
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
        info!("Multiexp on {} ({} GB, {} CUs): {} terms per pass", device.name(),
              device.memory() >> 30, device.compute_units(), n);
        Ok(SingleMultiexpKernel { program, n, curve, maybe_abort, _phantom: std::marker::PhantomData })
    }

    /// sum_i exponents[i] * bases[i].  Bases go over in their GPU form
    /// ([x, y], identity all zero, as multiexp.rs:152 builds it); exponents are
    /// canonical `BigInt`s; any length (the engine splits into passes).
    pub fn multiexp(
        &self, bases: &[G], exponents: &[<G::Scalar as PrimeField>::Repr],
    ) -> EcResult<G::Curve> {
        assert_eq!(bases.len(), exponents.len());
        require(&self.program, sys::ECG_KIND_MULTIEXP, self.curve)?;
        let repr: Vec<_> = bases.iter().map(GpuRepr::to_gpu_repr).collect();
        let mut acc = G::Curve::zero();
        let (cb, user) = abort_hook(&self.maybe_abort);
        check(unsafe {
            sys::ecg_msm(self.program.ctx(), self.curve, repr.as_ptr() as *const u64,
                         exponents.as_ptr() as *const u64, exponents.len(),
                         &mut acc as *mut G::Curve as *mut u64, cb, user)
        })?;
        Ok(acc)
    }
}

/// One multiexp kernel per device.
pub struct MultiexpKernel<'a, G>
where G: GpuCurveAffine
{
    kernels: Vec<SingleMultiexpKernel<'a, G>>,
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
        Ok(MultiexpKernel { kernels })
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
        let per_device = (exps.len() + self.kernels.len() - 1) / self.kernels.len().max(1);
        if per_device == 0 {
            return;
        }
        let ranges = bases.chunks(per_device).zip(exps.chunks(per_device));
        for ((kern, (bs, es)), slot) in self.kernels.iter_mut().zip(ranges).zip(results.iter_mut()) {
            let error = error.clone();
            scope.execute(move || {
                let mut partial = G::Curve::zero();
                for (b, e) in bs.chunks(kern.n).zip(es.chunks(kern.n)) {
                    if error.read().unwrap().is_err() {
                        return;
                    }
                    match kern.multiexp(b, e) {
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
    /// per-device partials are added on the host (multiexp.rs:372-400).
    pub fn multiexp(
        &mut self, pool: &Worker, bases_arc: Arc<Vec<G>>,
        exps: Arc<Vec<<G::Scalar as PrimeField>::Repr>>, skip: usize,
    ) -> EcResult<G::Curve> {
        let bases = &bases_arc[skip..(skip + exps.len())];
        let exps = &exps[..];
        let mut partials = vec![G::Curve::zero(); self.kernels.len()];
        let error = Arc::new(RwLock::new(Ok(())));
        pool.scoped(|s| self.parallel_multiexp(s, bases, exps, &mut partials, error.clone()));
        Arc::try_unwrap(error).expect("only one ref left").into_inner().unwrap()?;
        Ok(partials.into_iter().fold(G::Curve::zero(), |acc, p| acc + p))
    }

    /// Kernels (devices) in use.
    pub fn num_kernels(&self) -> usize {
        self.kernels.len()
    }
}
