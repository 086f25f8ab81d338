"""Run the 2^N MSM a few times (profiling target, dev tool).
Usage: python tools/msm_once.py [log_n] [reps] [prepared: 0|1] [curve]"""
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "0g-ec-gpu_amd"))
import ecgpu
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
prog = ecgpu.program(ecgpu.Device(0))
n = 1 << log_n
curve = sys.argv[4] if len(sys.argv) > 4 else "bls12_381"
rng = np.random.default_rng(7)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); E[:, 3] &= np.uint64(2**62 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
d_b = ecgpu.gen_bases_dev(prog, curve, 12345, 678910, n)
if len(sys.argv) > 3 and sys.argv[3] == "1":
    d_b = ecgpu.prepare_bases(prog, curve, d_b, n)
for _ in range(reps):
    ecgpu.msm_dev(prog, curve, d_b, d_e, n)
print("done")
