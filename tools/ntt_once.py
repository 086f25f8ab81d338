"""Run the 2^N Fr NTT a few times on device-resident data (profiling target, dev tool).
Usage: python tools/ntt_once.py [log_n] [reps] [bls12_381_fr|bn254_fr]"""
import os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
field = sys.argv[3] if len(sys.argv) > 3 else "bls12_381_fr"
if field == "bls12_381_fr":
    R, gen, adic = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001, 7, 32
else:
    R, gen, adic = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001, 5, 28
w = pow(gen, (R - 1) >> adic, R)
for _ in range(log_n, adic):
    w = w * w % R
x = w * (1 << 256) % R
om = np.array([(x >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
prog = ecgpu.program(ecgpu.Device(0))
a = np.random.default_rng(1).integers(0, 2**64, size=(1 << log_n, 4), dtype=np.uint64)
a[:, 3] &= np.uint64(2**61 - 1)
d = ecgpu.DeviceBuffer.upload(prog, a)
for _ in range(reps):
    ecgpu.fft_dev(prog, field, d, om, log_n)
print("done")
