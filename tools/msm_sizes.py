"""Time the prepared-bases MSM at the per-rank shard sizes of the strong-
scaling bench (2^26 / N terms for N = 1, 2, 4, 8) on one GPU (dev tool): the
per-rank work of an N-GPU run without the RCCL all-gather (144 B per rank).
Usage: python tools/msm_sizes.py [log_n ...]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

logs = [int(x) for x in sys.argv[1:]] or [23, 24, 25, 26]
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(7)
for ln in logs:
    n = 1 << ln
    E = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    E[:, 3] &= np.uint64(2**62 - 1)
    d_e = ecgpu.DeviceBuffer.upload(prog, E)
    d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 12345, 678910, n)
    pb = ecgpu.prepare_bases(prog, "bls12_381", d_b, n)
    d_b.free()
    for _ in range(2):
        res = ecgpu.msm_dev(prog, "bls12_381", pb, d_e, n)
    best, acc = 1e9, 1e9
    for _ in range(5):
        t = time.perf_counter()
        ecgpu.msm_dev(prog, "bls12_381", pb, d_e, n)
        best = min(best, time.perf_counter() - t)
        acc = min(acc, prog.kernel_time("msm_accumulate")[0])
    print(json.dumps({"log_n": ln, "ranks_at_2^26": 1 << (26 - ln), "ms": best * 1e3, "acc_ms": acc,
                      "point_adds_per_s": n / best,
                      "digest": hashlib.sha256(np.asarray(res).tobytes()).hexdigest()[:16]}), flush=True)
    pb.free()
    d_e.free()
