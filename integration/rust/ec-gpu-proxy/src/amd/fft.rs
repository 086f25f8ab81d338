//! Radix FFT over a prime field on MI355X (feature `amd`): the public API of
//! ec-gpu-proxy/src/fft.rs (SingleFftKernel 19-135, FftKernel 139-246) over
//! libecgpu.so's LDS Stockham NTT (ecg_fft / ecg_fft_many).

use ag_types::GpuName;
use ark_ff::Field;
use ec_gpu_program::{EcError, EcResult};
use ecgpu_sys as sys;
use log::{error, info};
use rust_gpu_tools::Program;

use super::{abort_hook, check, field_id, require, MaybeAbort};

/// FFT on one device.
pub struct SingleFftKernel<'a, F>
where F: Field + GpuName
{
    program: Program,
    maybe_abort: Option<&'a (dyn Fn() -> bool + Send + Sync)>,
    _phantom: std::marker::PhantomData<F>,
}

impl<'a, F: Field + GpuName> SingleFftKernel<'a, F> {
    /// A kernel on `program`'s device; `maybe_abort` is polled before each
    /// NTT pass and a `true` ends the call with `EcError::Aborted`.
    pub fn create(
        program: Program,
        maybe_abort: Option<&'a (dyn Fn() -> bool + Send + Sync)>,
    ) -> EcResult<Self> {
        Ok(SingleFftKernel { program, maybe_abort, _phantom: Default::default() })
    }

    /// `input` (2^log_n Montgomery elements, natural order) is replaced by its
    /// DFT at `omega`: a[k] = sum_j a[j] omega^(jk), no 1/n scaling.
    pub fn radix_fft(
        &mut self, input: &mut [F], omega: &F, log_n: u32,
    ) -> EcResult<()> {
        assert_eq!(input.len(), 1usize << log_n, "input length must be 2^log_n");
        let field = field_id::<F>()?;
        require(&self.program, sys::ECG_KIND_FFT, field)?;
        let (cb, user) = abort_hook(&self.maybe_abort);
        check(unsafe {
            sys::ecg_fft(self.program.ctx(), field, input.as_mut_ptr() as *mut u64,
                         omega as *const F as *const u64, log_n, cb, user)
        })
    }
}

/// One FFT kernel per device.
pub struct FftKernel<'a, F>
where F: Field + GpuName
{
    kernels: Vec<SingleFftKernel<'a, F>>,
}

impl<'a, F> FftKernel<'a, F>
where F: Field + GpuName
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
            match SingleFftKernel::<F>::create(program, maybe_abort) {
                Ok(k) => kernels.push(k),
                Err(e) => error!("Cannot initialize kernel for device '{}'! Error: {}", name, e),
            }
        }
        if kernels.is_empty() {
            return Err(EcError::Simple("No working GPUs found!"));
        }
        info!("FFT: {} MI355X context(s)", kernels.len());
        Ok(Self { kernels })
    }

    /// One transform on the first device.
    pub fn radix_fft(
        &mut self, input: &mut [F], omega: &F, log_n: u32,
    ) -> EcResult<()> {
        self.kernels[0].radix_fft(input, omega, log_n)
    }

    /// Many transforms over every device: ceil(count / #devices) consecutive
    /// transforms per device, each device on its own host thread inside the
    /// engine, the first error returned.
    pub fn radix_fft_many(
        &mut self, inputs: &mut [&mut [F]], omegas: &[F], log_ns: &[u32],
    ) -> EcResult<()> {
        assert!(inputs.len() == omegas.len() && inputs.len() == log_ns.len());
        for (input, &log_n) in inputs.iter().zip(log_ns) {
            assert_eq!(input.len(), 1usize << log_n, "input length must be 2^log_n");
        }
        let field = field_id::<F>()?;
        for k in &self.kernels {
            require(&k.program, sys::ECG_KIND_FFT, field)?;
        }
        let mut ctxs: Vec<_> = self.kernels.iter().map(|k| k.program.ctx()).collect();
        let mut ptrs: Vec<*mut u64> = inputs.iter_mut().map(|s| s.as_mut_ptr() as *mut u64).collect();
        let (cb, user) = abort_hook(&self.kernels[0].maybe_abort);
        check(unsafe {
            sys::ecg_fft_many(ctxs.as_mut_ptr(), ctxs.len() as i32, field, ptrs.as_mut_ptr(),
                              omegas.as_ptr() as *const u64, log_ns.as_ptr(), ptrs.len(), cb, user)
        })
    }
}
