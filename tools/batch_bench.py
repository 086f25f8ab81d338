"""Timing of the batched multi-line MSM on the shape of ag-cuda-ec/benches/
amt.rs (LOG_N = 10: LENGTH = 2^21 scalars, 10 lines of bases, 2^7 .. 2^11
chunks per line).  Dev tool; prints one JSON line per configuration.
Usage: python tools/batch_bench.py [log_n] [--cycled] [--prepared] [--chunks=K]
--prepared: bases converted once (upload_multiexp_bases); --chunks=K: only
that chunk count."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
cycled = "--cycled" in sys.argv
L = 1 << (2 * log_n + 1)
lines = log_n
prog = ecgpu.program(ecgpu.Device(0))
rng = np.random.default_rng(1)
if cycled:  # random_input_by_cycle(LENGTH, 73)
    meta = rng.integers(0, 2**64, size=(73, 4), dtype=np.uint64)
    meta[:, 3] &= np.uint64(2**62 - 1)
    E = np.ascontiguousarray(np.resize(meta, (L, 4)))
else:
    E = rng.integers(0, 2**64, size=(L, 4), dtype=np.uint64)
    E[:, 3] &= np.uint64(2**62 - 1)
d_b = ecgpu.gen_bases_dev(prog, "bls12_381", 99, 12345, L * lines)
if "--prepared" in sys.argv:
    d_b = ecgpu.prepare_bases(prog, "bls12_381", d_b, L * lines)
d_e = ecgpu.DeviceBuffer.upload(prog, E)
only = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--chunks=")]
for chunks in only or [1 << gdeg for gdeg in range(7, 12)]:
    ecgpu.multiple_multiexp(prog, d_b, (d_e, L), chunks)
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        ecgpu.multiple_multiexp(prog, d_b, (d_e, L), chunks)
        best = min(best, time.perf_counter() - t)
    acc = prog.kernel_time("msm_accumulate")[0]
    terms = L * lines
    print(json.dumps({"lines": lines, "line_len": L, "chunks": chunks, "tasks": lines * chunks,
                      "chunk_len": L // chunks, "ms": round(best * 1e3, 2), "acc_ms": round(acc, 2),
                      "terms_per_s": terms / best, "cycled": cycled, "prepared": "--prepared" in sys.argv}), flush=True)
