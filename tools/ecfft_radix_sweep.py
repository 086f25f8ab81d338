"""EC-FFT stage-radix sweep (dev tool): device-resident ecg_ec_fft_dev for each
size and each largest log-radix (ecg_ec_fft_set_radix: 1 = radix-2 stages
only, 0 = the library's choice), same input, same output digest required.
Usage: python tools/ecfft_radix_sweep.py curve "0 1 2 ..." "log_n ..." [batch]"""
import hashlib
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

curve = sys.argv[1]
radices = [int(x) for x in sys.argv[2].split()]
sizes = [int(x) for x in sys.argv[3].split()]
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
cv = po.CURVES[curve]
lq = cv.fq.limbs64
prog = ecgpu.program(ecgpu.Device(0))
one = co.u64arr([cv.fq.to_mont(1)], lq)[0]
for log_n in sizes:
    n = 1 << log_n
    d_aff = ecgpu.gen_bases_dev(prog, curve, 3, 7, n * batch)
    aff = d_aff.read(shape=(n * batch, 2 * lq))
    d_aff.free()
    jac = np.ascontiguousarray(np.concatenate([aff, np.tile(one, (n * batch, 1))], axis=1))
    om = co.u64arr([cv.fr.to_mont(cv.fr.omega(n))], 4)[0]
    k = ecgpu.EcFftKernel.create([prog], curve)
    rec = {"curve": curve, "log_n": log_n, "batch": batch, "ms": {}}
    digests = set()
    for rx in radices:
        ecgpu.ec_fft_set_radix(rx)
        if batch == 1:
            d = ecgpu.DeviceBuffer.upload(prog, jac)
            ecgpu.ec_fft_dev(prog, curve, d, om, log_n)  # warm-up (tables, workspace)
            best = 1e9
            for _ in range(3):
                d.write(jac)
                t = time.perf_counter()
                ecgpu.ec_fft_dev(prog, curve, d, om, log_n)
                best = min(best, time.perf_counter() - t)
            out = d.read(shape=jac.shape)
            d.free()
        else:  # radix_ec_fft_many over `batch` equal inputs (host buffers): one batched transform
            xs = [np.ascontiguousarray(jac[i * n:(i + 1) * n]) for i in range(batch)]
            k.radix_ec_fft_many([x.copy() for x in xs], [om] * batch, [log_n] * batch)
            best = 1e9
            for _ in range(3):
                ys = [x.copy() for x in xs]
                t = time.perf_counter()
                k.radix_ec_fft_many(ys, [om] * batch, [log_n] * batch)
                best = min(best, time.perf_counter() - t)
            out = np.concatenate(ys)
        digests.add(hashlib.sha256(out.tobytes()).hexdigest()[:16])
        rec["ms"][rx] = round(best * 1e3, 3)
    ecgpu.ec_fft_set_radix(0)
    rec["same_output"] = len(digests) == 1
    print(json.dumps(rec), flush=True)
