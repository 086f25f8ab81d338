"""EC-FFT timing (dev tool): device-resident ecg_ec_fft_dev at several sizes,
per-stage kernel time from the library's HIP-event timer, and the oracle's
serial_ec_fft (16 host threads) on a small size for scale.
Usage: python tools/ecfft_bench.py [curve] [log_n ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd"), os.path.join(ROOT, "oracle")]
import coracle as co  # noqa: E402
import ecgpu  # noqa: E402
import py_oracle as po  # noqa: E402

curve = sys.argv[1] if len(sys.argv) > 1 else "bls12_381"
sizes = [int(x) for x in sys.argv[2:]] or [10, 12, 14, 16, 18]
cid = ecgpu.CURVE_NAMES[curve]
cv = po.CURVES[curve]
lq = cv.fq.limbs64
prog = ecgpu.program(ecgpu.Device(0))
one = co.u64arr([cv.fq.to_mont(1)], lq)[0]
for log_n in sizes:
    n = 1 << log_n
    d_aff = ecgpu.gen_bases_dev(prog, curve, 3, 7, n)
    aff = d_aff.read(shape=(n, 2 * lq))
    jac = np.ascontiguousarray(np.concatenate([aff, np.tile(one, (n, 1))], axis=1))
    om = co.u64arr([cv.fr.to_mont(cv.fr.omega(n))], 4)[0]
    d = ecgpu.DeviceBuffer.upload(prog, jac)
    ecgpu.ec_fft_dev(prog, curve, d, om, log_n)  # warm-up
    best = 1e9
    for _ in range(2):
        d.write(jac)
        t = time.perf_counter()
        ecgpu.ec_fft_dev(prog, curve, d, om, log_n)
        best = min(best, time.perf_counter() - t)
    st_ms, st_n = prog.kernel_time("ecfft_stage")
    rec = {"curve": curve, "log_n": log_n, "ms": round(best * 1e3, 3), "stage_ms": round(st_ms, 3),
           "stages": st_n, "butterflies_per_s": (n // 2) * log_n / best}
    if log_n <= 12:
        t = time.perf_counter()
        co.serial_ec_fft(cid, jac, om, log_n, nthreads=16)
        rec["cpu_oracle_16t_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    print(json.dumps(rec), flush=True)
