"""A/B of MSM tunables (AB_CURVE=bn254 for the other G1 curve; ECGPU_LIB=<lib> as a config
selects another in-tree build) (env vars read once per process -> one subprocess per
config, interleaved rounds).  Dev tool: prints per-kernel times from the
library's HIP-event timer and the end-to-end ms per 2^N MSM."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOG = int(sys.argv[1]) if len(sys.argv) > 1 else 26
CONFIGS = [dict(x.split("=") for x in c.split(",")) if c else {} for c in (sys.argv[2:] or [""])]
CODE = r'''
import sys, time, json, numpy as np
sys.path.insert(0, "%s/0g-ec-gpu_amd")
import ecgpu
prog = ecgpu.program(ecgpu.Device(0))
n = 1 << %d
rng = np.random.default_rng(7)
E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); E[:, 3] &= np.uint64(2**62 - 1)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
CV = "%s"
d_b = ecgpu.prepare_bases(prog, CV, ecgpu.gen_bases_dev(prog, CV, 12345, 678910, n), n)
for _ in range(2): ecgpu.msm_dev(prog, CV, d_b, d_e, n)
best = 1e9; acc = 1e9
for _ in range(5):
    t = time.perf_counter(); out = ecgpu.msm_dev(prog, CV, d_b, d_e, n); best = min(best, time.perf_counter() - t)
    acc = min(acc, prog.kernel_time("msm_accumulate")[0])
import hashlib
print(json.dumps({"ms": best * 1e3, "acc_ms": acc, "result": hashlib.sha256(out.tobytes()).hexdigest()[:16]}))
''' % (ROOT, LOG, os.environ.get("AB_CURVE", "bls12_381"))
for rnd in range(2):
    for cfg in CONFIGS:
        env = dict(os.environ, **cfg)
        out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
        print(rnd, cfg, out.stdout.strip()[-200:], out.stderr.strip()[-300:] if out.returncode else "", flush=True)
