"""A/B of the G2 EC-FFT butterfly field (dev tool): ECG_ECFFT_RR=1 (reduced-
radix Fq2, default) against ECG_ECFFT_RR=0 (32-bit-limb Fq2), one subprocess
per config; prints ms per radix_ec_fft and a digest of the output (the two
must agree).  Parity is tests/test_gpu_g2.py's linearity test.
Usage: python tools/ecfft_g2_ab.py [curve] [log_n ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CURVE = sys.argv[1] if len(sys.argv) > 1 else "bls12_381_g2"
SIZES = [int(x) for x in sys.argv[2:]] or [10, 12]
CODE = r'''
import sys, time, hashlib, json, numpy as np
sys.path[:0] = ["%s/0g-ec-gpu_amd", "%s/oracle"]
import ecgpu, coracle as co, py_oracle as po
curve = "%s"
cv = po.CURVES[curve[:-3]]
lq = 2 * cv.fq.limbs64
one = np.zeros(lq, dtype=np.uint64)
one[:cv.fq.limbs64] = co.u64arr([cv.fq.to_mont(1)], cv.fq.limbs64)[0]
prog = ecgpu.program(ecgpu.Device(0))
k = ecgpu.EcFftKernel.create([prog], curve)
out = {}
for log_n in %s:
    n = 1 << log_n
    aff = ecgpu.gen_bases_dev(prog, curve, 3, 7, n).read(shape=(n, 2 * lq))
    base = np.ascontiguousarray(np.concatenate([aff, np.tile(one, (n, 1))], axis=1))
    om = co.u64arr([cv.fr.to_mont(cv.fr.omega(n))], 4)[0]
    best = 1e9
    for _ in range(3):
        jac = base.copy()
        t = time.perf_counter(); k.radix_ec_fft(jac, om, log_n); best = min(best, time.perf_counter() - t)
    out[log_n] = {"ms": best * 1e3, "digest": hashlib.sha256(jac.tobytes()).hexdigest()[:16]}
print(json.dumps(out))
''' % (ROOT, ROOT, CURVE, SIZES)
for rr in ("1", "0"):
    p = subprocess.run([sys.executable, "-c", CODE], env=dict(os.environ, ECG_ECFFT_RR=rr), capture_output=True,
                       text=True, timeout=900)
    print(f"ECG_ECFFT_RR={rr}", p.stdout.strip() if p.returncode == 0 else p.stderr.strip()[-600:], flush=True)
