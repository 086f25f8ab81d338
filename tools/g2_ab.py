"""A/B of the G2 MSM pipeline field (dev tool): ECG_MSM_RR=1 (reduced-radix
Fq2, default) against ECG_MSM_RR=0 (32-bit-limb Fq2), one subprocess per
config, interleaved rounds; prints ms per 2^N G2 MSM over prepared bases,
the accumulate kernel's HIP-event time, and whether both configs agree.
Usage: python tools/g2_ab.py [log_n] [curve]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOG = int(sys.argv[1]) if len(sys.argv) > 1 else 20
CURVE = sys.argv[2] if len(sys.argv) > 2 else "bls12_381_g2"
CODE = r'''
import sys, time, json, hashlib, numpy as np
sys.path.insert(0, "%s/0g-ec-gpu_amd")
import ecgpu
prog = ecgpu.program(ecgpu.Device(0))
n = 1 << %d
rng = np.random.default_rng(11)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); E[:, 3] &= np.uint64(2**60 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
d_b = ecgpu.gen_bases_dev(prog, "%s", 12345, 678910, n)
d_p = ecgpu.prepare_bases(prog, "%s", d_b, n)
out = ecgpu.msm_dev(prog, "%s", d_p, d_e, n)
best = 1e9; acc = 1e9
for _ in range(3):
    t = time.perf_counter(); out = ecgpu.msm_dev(prog, "%s", d_p, d_e, n); best = min(best, time.perf_counter() - t)
    acc = min(acc, prog.kernel_time("msm_accumulate")[0])
print(json.dumps({"ms": best * 1e3, "acc_ms": acc, "out": hashlib.sha256(out.tobytes()).hexdigest()[:16]}))
''' % (ROOT, LOG, CURVE, CURVE, CURVE, CURVE)
res = {}
for rnd in range(2):
    for rr in ("1", "0"):
        env = dict(os.environ, ECG_MSM_RR=rr)
        p = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
        line = p.stdout.strip().splitlines()[-1] if p.returncode == 0 else p.stderr.strip()[-400:]
        print(rnd, f"ECG_MSM_RR={rr}", line, flush=True)
        if p.returncode == 0:
            res[rr] = json.loads(line)["out"]
print("results agree:", len(set(res.values())) == 1)
