//! FFT over elliptic-curve points ("FFTg") on MI355X (feature `amd`): the
//! public API of ec-gpu-proxy/src/ec_fft.rs (SingleEcFftKernel 18-160,
//! EcFftKernel 164-280) over libecgpu.so's windowed-GLV stages (ecg_ec_fft).

use ag_types::{GpuCurveAffine, GpuName};
use ark_ff::Field;
use ec_gpu_program::{EcError, EcResult};
use ecgpu_sys as sys;
use log::{error, info};
use rust_gpu_tools::Program;

use super::{abort_hook, check, curve_id, require, MaybeAbort};

/// EC-FFT on one device.
pub struct SingleEcFftKernel<'a, G>
where
    G: GpuCurveAffine,
    G::Scalar: Field + GpuName,
{
    program: Program,
    maybe_abort: Option<&'a (dyn Fn() -> bool + Send + Sync)>,
    _phantom: std::marker::PhantomData<G::Scalar>,
}

impl<'a, G: GpuCurveAffine> SingleEcFftKernel<'a, G>
where G::Scalar: Field + GpuName
{
    /// A kernel on `program`'s device; `maybe_abort` is polled before the
    /// transform starts.
    pub fn create(
        program: Program,
        maybe_abort: Option<&'a (dyn Fn() -> bool + Send + Sync)>,
    ) -> EcResult<Self> {
        // the engine reads and writes `G::Curve` as [X, Y, Z] in place
        ecgpu_ark::require_projective_xyz::<G>().map_err(EcError::Simple)?;
        Ok(SingleEcFftKernel { program, maybe_abort, _phantom: Default::default() })
    }

    /// `input` (2^log_n projective points, natural order) is replaced by
    /// P_k = sum_j omega^(jk) P_j, written back normalised.
    pub fn radix_ec_fft(
        &mut self, input: &mut [G::Curve], omega: &G::Scalar, log_n: u32,
    ) -> EcResult<()> {
        assert_eq!(input.len(), 1usize << log_n, "input length must be 2^log_n");
        ecgpu_ark::require_projective_xyz::<G>().map_err(EcError::Simple)?;
        let curve = curve_id::<G>()?;
        require(&self.program, sys::ECG_KIND_EC_FFT, curve)?;
        let (cb, user) = abort_hook(&self.maybe_abort);
        check(unsafe {
            sys::ecg_ec_fft(self.program.ctx(), curve, input.as_mut_ptr() as *mut u64,
                            omega as *const G::Scalar as *const u64, log_n, cb, user)
        })
    }
}

/// One EC-FFT kernel per device.
pub struct EcFftKernel<'a, G>
where
    G: GpuCurveAffine,
    G::Scalar: Field + GpuName,
{
    kernels: Vec<SingleEcFftKernel<'a, G>>,
}

impl<'a, G> EcFftKernel<'a, G>
where
    G: GpuCurveAffine,
    G::Scalar: Field + GpuName,
{
    /// One kernel per program.
    pub fn create(programs: Vec<Program>) -> EcResult<Self> {
        Self::create_optional_abort(programs, None)
    }

    /// One kernel per program, each polling `maybe_abort`.
    pub fn create_with_abort(
        programs: Vec<Program>,
        maybe_abort: &'a (dyn Fn() -> bool + Send + Sync),
    ) -> EcResult<Self> {
        Self::create_optional_abort(programs, Some(maybe_abort))
    }

    fn create_optional_abort(programs: Vec<Program>, maybe_abort: MaybeAbort<'a>) -> EcResult<Self> {
        let mut kernels = Vec::with_capacity(programs.len());
        for program in programs {
            let name = program.device_name().to_string();
            match SingleEcFftKernel::<G>::create(program, maybe_abort) {
                Ok(k) => kernels.push(k),
                Err(e) => error!("Cannot initialize kernel for device '{}'! Error: {}", name, e),
            }
        }
        if kernels.is_empty() {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        info!("FFTg: {} MI355X context(s)", kernels.len());
        Ok(Self { kernels })
    }

    /// One transform on the first device.
    pub fn radix_ec_fft(
        &mut self, input: &mut [G::Curve], omega: &G::Scalar, log_n: u32,
    ) -> EcResult<()> {
        self.kernels[0].radix_ec_fft(input, omega, log_n)
    }

    /// Many transforms over every device, ceil(count / #devices) per device,
    /// the first error returned.
    pub fn radix_ec_fft_many(
        &mut self, inputs: &mut [&mut [G::Curve]], omegas: &[G::Scalar],
        log_ns: &[u32],
    ) -> EcResult<()> {
        assert!(inputs.len() == omegas.len() && inputs.len() == log_ns.len());
        for (input, &log_n) in inputs.iter().zip(log_ns) {
            assert_eq!(input.len(), 1usize << log_n, "input length must be 2^log_n");
        }
        ecgpu_ark::require_projective_xyz::<G>().map_err(EcError::Simple)?;
        let curve = curve_id::<G>()?;
        for k in &self.kernels {
            require(&k.program, sys::ECG_KIND_EC_FFT, curve)?;
        }
        let mut ctxs: Vec<_> = self.kernels.iter().map(|k| k.program.ctx()).collect();
        let mut ptrs: Vec<*mut u64> = inputs.iter_mut().map(|s| s.as_mut_ptr() as *mut u64).collect();
        let (cb, user) = abort_hook(&self.kernels[0].maybe_abort);
        check(unsafe {
            sys::ecg_ec_fft_many(ctxs.as_mut_ptr(), ctxs.len() as i32, curve, ptrs.as_mut_ptr(),
                                 omegas.as_ptr() as *const u64, log_ns.as_ptr(), ptrs.len(), cb, user)
        })
    }
}
