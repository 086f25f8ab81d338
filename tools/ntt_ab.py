"""A/B timing of NTT variants in one process (dev tool): ECG_NTT_VARIANT is read
once per process, so each variant runs in its own subprocess, interleaved."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, time, json, numpy as np
sys.path.insert(0, "%s/0g-ec-gpu_amd"); sys.path.insert(0, "%s/oracle")
import ecgpu, coracle as co, py_oracle as po
f = po.BLS12_381_FR
prog = ecgpu.program(ecgpu.Device(0))
res = {}
for log_n in (20, 24):
    n = 1 << log_n
    a = np.random.default_rng(log_n).integers(0, 2**62, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64(2**60 - 1)
    om = co.u64arr([f.to_mont(f.omega(n))], 4)[0]
    d = ecgpu.DeviceBuffer.upload(prog, a)
    for _ in range(3): ecgpu.fft_dev(prog, "bls12_381_fr", d, om, log_n)
    best = 1e9
    for _ in range(10):
        t = time.perf_counter(); ecgpu.fft_dev(prog, "bls12_381_fr", d, om, log_n); best = min(best, time.perf_counter() - t)
    ms, cnt = prog.kernel_time("ntt_pass")
    ok = None
    if log_n <= 24:
        d.write(a); ecgpu.fft_dev(prog, "bls12_381_fr", d, om, log_n)
        ok = bool((d.read(shape=(n, 4)) == co.parallel_fft(0, a, om, log_n, 3)).all())
    res[log_n] = {"ms": best * 1e3, "kernel_ms": ms, "passes": cnt, "ok": ok}
    d.free()
print(json.dumps(res))
''' % (ROOT, ROOT)
# configs: "KEY=VAL,KEY=VAL" env sets (default: the radix / pass-count variants)
CONFIGS = [dict(x.split("=") for x in c.split(",")) if c else {} for c in sys.argv[1:]] or [
    dict(ECG_NTT_VARIANT=v, ECG_NTT_MAXDEG=md) for v, md in (("1", "8"), ("2", "8"), ("2", "10"), ("2", "12"))]
for rnd in range(2):
    for cfg in CONFIGS:
        env = dict(os.environ, **cfg)
        out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
        print(cfg, "round", rnd, out.stdout.strip()[-600:], out.stderr.strip()[-300:] if out.returncode else "", flush=True)
