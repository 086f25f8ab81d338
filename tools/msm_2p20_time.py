"""Best-of-30 prepared 2^20 MSM on both curves plus the cost of one msm_chunk_size query (dev tool)."""
import os, sys, time
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd"), os.path.join(ROOT, "oracle"), ROOT]
import ecgpu, bench
prog = ecgpu.program(ecgpu.Device(0))
for cv, r in (("bls12_381", bench.R_BLS), ("bn254", bench.R_BN)):
    n = 1 << 20
    d_e = ecgpu.DeviceBuffer.upload(prog, bench.rand_scalars(np.random.default_rng(1), n, r))
    raw = ecgpu.gen_bases_dev(prog, cv, 3, 5, n)
    prep = ecgpu.prepare_bases(prog, cv, raw, n)
    ecgpu.msm_dev(prog, cv, prep, d_e, n)
    ts = []
    for _ in range(30):
        t = time.perf_counter(); ecgpu.msm_dev(prog, cv, prep, d_e, n); ts.append(time.perf_counter() - t)
    t = time.perf_counter()
    for _ in range(200): prog.msm_chunk_size(cv)
    q = (time.perf_counter() - t) / 200
    print(f"{cv} 2^20 best {min(ts)*1e3:.3f} ms median {sorted(ts)[15]*1e3:.3f} ms; msm_chunk_size call {q*1e6:.1f} us", flush=True)
