"""NTT 2^24 pass times in different surroundings (dev tool): why is the NTT
slower inside bench.py than alone?  Modes (argv[1]):
  alone    -- fresh context, NTT only
  frag     -- after allocating / freeing the MSM-sized buffers bench.py holds
  hold     -- while the MSM-sized buffers stay allocated (no MSM run)
  msm      -- right after 8 back-to-back 2^26 MSMs (power / clock state)
Prints per-pass kernel ms (HIP events) averaged over the reps."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "alone"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
w = pow(7, (R - 1) >> 32, R)
for _ in range(24, 32):
    w = w * w % R
x = w * (1 << 256) % R
om = np.array([(x >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
prog = ecgpu.program(ecgpu.Device(0))
held = []
if mode in ("frag", "hold", "msm"):
    n = 1 << 26
    rng = np.random.default_rng(7)
    E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    E[:, 3] &= np.uint64(2**62 - 1)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 12345, 678910, n)
    d_p = ecgpu.prepare_bases(prog, "bls12_381", d_b, n)
    ecgpu.msm_dev(prog, "bls12_381", d_p, d_e, n)  # grows the MSM workspace
    if mode == "msm":
        for _ in range(8):
            ecgpu.msm_dev(prog, "bls12_381", d_p, d_e, n)
    if mode == "frag":
        d_e.free()
        d_b.free()
        d_p.free()
    else:
        held = [d_e, d_b, d_p]
a = np.random.default_rng(1).integers(0, 2**64, size=(1 << 24, 4), dtype=np.uint64)
a[:, 3] &= np.uint64(2**62 - 1)
d = ecgpu.DeviceBuffer.upload(prog, a)
ecgpu.fft_dev(prog, "bls12_381_fr", d, om, 24)
tot, launches = 0.0, 0
t0 = time.perf_counter()
for _ in range(reps):
    ecgpu.fft_dev(prog, "bls12_381_fr", d, om, 24)
    ms, cnt = prog.kernel_time("ntt_pass")
    tot += ms
    launches += cnt
wall = (time.perf_counter() - t0) / reps
print(f"{mode}: wall {wall * 1e3:.3f} ms/ntt, kernels {tot / reps:.3f} ms/ntt, {tot / launches:.3f} ms/pass")
