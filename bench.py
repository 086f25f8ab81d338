#!/usr/bin/env python3
"""bench.py -- BLS12-381 G1 MSM point-adds/s @2^26 + Fr NTT elements/s @2^24 on MI355X.

Workload (BASELINE.json metric): one step = one G1 Pippenger MSM over 2^26
(base, scalar) terms, the terms sharded in contiguous ranges across the N
ranks (BASELINE config 4; at N=1 the whole 2^26 on one GPU), with the per-rank
partial sums all-gathered over RCCL and folded on the device.  The NTT leg
times one in-place 2^24 Fr NTT per rank per step (radix_fft_many: whole
transforms per GPU, no exchange) and is reported in the "ntt" object.

Inputs are synthetic and resident in HBM before the timed region:
bases P_i = (a + i*b) G generated on the GPU, scalars uniform < r (xoshiro/
numpy, seeded), NTT input uniform Fr.  `value` = total MSM terms / step time
(whole job).  Parity is checked every run: the MSM result against the
known-answer (sum s_i (a + i b) mod r) * G, the NTT against the CPU oracle's
parallel_fft at the full 2^24 size.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402  (product path: libecgpu.so, fails loudly if missing)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
MAD_PEAK_TLANE = 35.3          # measured v_mad_u64_u32 lane-ops/s (tools/mad_microbench.hip), T/s
BLS_R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
MSM_SEED = 0x35A00026
NTT_SEED = 0x0FF70024
KAT_A = 0x1234567890ABCDEF1122334455667788
KAT_B = 0x0FEDCBA987654321


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--msm-log", type=int, default=26)
    ap.add_argument("--ntt-log", type=int, default=24)
    ap.add_argument("--curve", default="bls12_381")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--msm-cpu-log", type=int, default=20)
    return ap.parse_args()


def u64(x: int, n: int = 4) -> np.ndarray:
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)], dtype=np.uint64)


def limbs_to_int(a) -> int:
    return sum(int(v) << (64 * i) for i, v in enumerate(np.asarray(a, dtype=np.uint64).ravel()))


def rand_scalars(rng: np.random.Generator, n: int, r: int, nbits: int) -> np.ndarray:
    """uniform in [0, r) by rejection (vectorised)."""
    out = np.empty((n, 4), dtype=np.uint64)
    top_mask = np.uint64((1 << (nbits - 192)) - 1)
    r_limbs = u64(r)
    filled = 0
    while filled < n:
        m = n - filled
        cand = rng.integers(0, 2**64, size=(m, 4), dtype=np.uint64)
        cand[:, 3] &= top_mask
        # lexicographic compare against r from the top limb
        lt = np.zeros(m, dtype=bool)
        eq = np.ones(m, dtype=bool)
        for k in (3, 2, 1, 0):
            lt |= eq & (cand[:, k] < r_limbs[k])
            eq &= cand[:, k] == r_limbs[k]
        ok = cand[lt]
        take = min(len(ok), m)
        out[filled:filled + take] = ok[:take]
        filled += take
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    cid = ecgpu.CURVE_NAMES[args.curve]
    fr_fid = ecgpu.CURVE_FR_FIELD[cid]
    lq = ecgpu.CURVE_FQ_LIMBS[cid]
    L = ecgpu.lib()
    prog = ecgpu.program(ecgpu.Device(local_rank))
    ctx = prog.handle

    # ------------------------------------------------------------ MSM inputs
    n_total = 1 << args.msm_log
    per = (n_total + world - 1) // world
    i0 = min(n_total, rank * per)
    n_loc = min(n_total, i0 + per) - i0
    r_int = BLS_R if cid == 0 else 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
    nbits = r_int.bit_length()
    rng = np.random.default_rng([MSM_SEED, rank])
    scal = rand_scalars(rng, n_loc, r_int, nbits)
    d_scal = torch.from_numpy(scal.view(np.uint8).reshape(-1)).to(dev)
    d_bases = torch.empty(n_loc * 2 * lq * 8, dtype=torch.uint8, device=dev)
    a_loc = (KAT_A + i0 * KAT_B) % r_int
    rc = L.ecg_gen_bases_dev(ctx, cid, ecgpu._ptr(u64(a_loc)), ecgpu._ptr(u64(KAT_B)), n_loc,
                             ctypes.c_void_p(d_bases.data_ptr()), None)
    ecgpu._check(rc, "gen_bases")
    d_part = torch.zeros(3 * lq, dtype=torch.int64, device=dev)
    d_gather = torch.zeros(world * 3 * lq, dtype=torch.int64, device=dev)
    out_host = np.zeros(3 * lq, dtype=np.uint64)

    def msm_step():
        if world == 1:
            ecgpu._check(L.ecg_msm_dev(ctx, cid, ctypes.c_void_p(d_bases.data_ptr()),
                                       ctypes.c_void_p(d_scal.data_ptr()), n_loc,
                                       out_host.ctypes.data_as(ctypes.c_void_p), 0, None), "msm")
            return
        ecgpu._check(L.ecg_msm_dev(ctx, cid, ctypes.c_void_p(d_bases.data_ptr()),
                                   ctypes.c_void_p(d_scal.data_ptr()), n_loc,
                                   ctypes.c_void_p(d_part.data_ptr()), 1, None), "msm")
        dist.all_gather_into_tensor(d_gather, d_part)  # RCCL over xGMI: world x 144 B
        torch.cuda.synchronize()
        ecgpu._check(L.ecg_point_sum_dev(ctx, cid, ctypes.c_void_p(d_gather.data_ptr()), world,
                                         ecgpu._ptr(out_host), None), "fold")

    # ------------------------------------------------------------ NTT inputs
    log_n = args.ntt_log
    n_ntt = 1 << log_n
    # omega = TWO_ADIC_ROOT^(2^(S - log n)) (ec-gpu-proxy/tests/fft.rs:16-24), Montgomery R = 2^256
    gen, two_adicity = (7, 32) if cid == 0 else (5, 28)
    omega = pow(gen, (r_int - 1) >> two_adicity, r_int)
    for _ in range(log_n, two_adicity):
        omega = omega * omega % r_int
    omega_m = u64(omega * (1 << 256) % r_int)
    nrng = np.random.default_rng([NTT_SEED, rank])
    ntt_in = rand_scalars(nrng, n_ntt, r_int, nbits)  # uniform < r; any value is a valid Montgomery form
    d_ntt = torch.from_numpy(ntt_in.view(np.uint8).reshape(-1)).to(dev)
    d_ntt_work = torch.empty_like(d_ntt)

    def ntt_step(buf):
        # in place; back-to-back steps transform the previous output (still uniform Fr data)
        ecgpu._check(L.ecg_fft_dev(ctx, fr_fid, ctypes.c_void_p(buf.data_ptr()), ecgpu._ptr(omega_m),
                                   log_n, None), "ntt")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ------------------------------------------------------------ MSM timing
    for _ in range(args.warmup):
        msm_step()
    barrier()
    t0 = time.perf_counter()
    acc_ms, acc_launch = 0.0, 0
    for _ in range(args.steps):
        msm_step()
        ms, cnt = prog.kernel_time("msm_accumulate")
        acc_ms += ms
        acc_launch += cnt
    barrier()
    msm_s = max_over_ranks(time.perf_counter() - t0) / args.steps
    acc_avg_ms = max_over_ranks(acc_ms / max(acc_launch, 1))

    # ------------------------------------------------------------ NTT timing
    d_ntt_work.copy_(d_ntt)
    for _ in range(args.warmup):
        ntt_step(d_ntt_work)
    barrier()
    t0 = time.perf_counter()
    pass_ms, pass_launch = 0.0, 0
    for _ in range(args.steps):
        ntt_step(d_ntt_work)
        ms, cnt = prog.kernel_time("ntt_pass")
        pass_ms += ms
        pass_launch += cnt
    barrier()
    ntt_s = max_over_ranks(time.perf_counter() - t0) / args.steps
    pass_avg_ms = max_over_ranks(pass_ms / max(pass_launch, 1))
    passes_per_ntt = pass_launch / args.steps
    # parity input: one fresh transform of the seeded input
    d_ntt_work.copy_(d_ntt)
    torch.cuda.synchronize()
    ntt_step(d_ntt_work)

    # ------------------------------------------------------------ oracle leg (rank 0, N = 1)
    # The CPU oracle (oracle/) is used here only as the checker and as the timed
    # CPU baseline, never on the measured path.
    checks = {}
    cpu_baseline = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle as co
        # MSM known answer: sum_i s_i (a + i b) mod r, times G  (SURVEY §8c KAT)
        kat = co.kat_scalar(cid, a_loc, KAT_B, scal, nthreads=args.cpu_threads)
        want = co.jac_to_affine(cid, co.gen_mul(cid, kat))
        got = co.jac_to_affine(cid, out_host)
        checks["msm_kat_2^%d" % args.msm_log] = bool(want is not None and got is not None and (want == got).all())
        # NTT: GPU result vs CPU parallel_fft (fft_cpu.rs:59-111) at the full size, bit-exact
        gpu_out = d_ntt_work.cpu().numpy().view(np.uint64).reshape(-1, 4)
        lt = min(4, log_n)
        t_cpu = time.perf_counter()
        ref = co.parallel_fft(fr_fid, ntt_in, omega_m, log_n, lt)
        ntt_cpu_s = time.perf_counter() - t_cpu
        checks["ntt_vs_parallel_fft_2^%d" % log_n] = bool((gpu_out == ref).all())
        # CPU baseline: multiexp_cpu restatement on a bounded sample of the same workload
        ns = 1 << args.msm_cpu_log
        sb = co.gen_bases(cid, 3, 5, ns, nthreads=args.cpu_threads)
        ss = np.ascontiguousarray(scal[:ns]) if ns <= n_loc else rand_scalars(rng, ns, r_int, nbits)
        t_cpu = time.perf_counter()
        co.multiexp_cpu(cid, sb, ss, nthreads=args.cpu_threads)
        cpu_s = time.perf_counter() - t_cpu
        cpu_baseline = {
            "value": ns / cpu_s, "unit": "point-adds/s", "cores": args.cpu_threads, "kind": "port",
            "sample": f"multiexp_cpu restatement (oracle/oracle.c, c=ceil(ln N), windows in parallel) on "
                      f"2^{args.msm_cpu_log} terms of the same generator: {cpu_s:.2f} s wall",
            "ntt": {"value": n_ntt / ntt_cpu_s, "unit": "elements/s", "cores": 1 << lt, "kind": "port",
                    "sample": f"parallel_fft restatement at the full 2^{log_n}: {ntt_cpu_s:.2f} s wall"},
        }

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ------------------------------------------------------------ report
    msm_bytes_per_term = 2 * lq * 8 + 32  # 96 B affine + 32 B scalar (BLS12-381), SURVEY §8(d)
    acc_achieved = msm_bytes_per_term * n_loc / (acc_avg_ms / 1e3) / 1e9
    ntt_achieved = 64 * n_ntt / (pass_avg_ms / 1e3) / 1e9
    line = {
        "metric": "BLS12-381 G1 MSM point-adds/sec @2^26 + Fr NTT elements/sec @2^24"
        if cid == 0 else "BN254 G1 MSM point-adds/sec + Fr NTT elements/sec",
        "value": n_total / msm_s,
        "unit": "point-adds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": msm_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32 limbs (mod-p int, v_mad_u64_u32)",
        "data": "synthetic (bases (a+i*b)G on GPU, scalars uniform < r, seeded)",
        "config": {"workload": f"{args.curve} G1 MSM 2^{args.msm_log} terms sharded over {world} GPU(s) "
                               f"+ Fr NTT 2^{log_n} per GPU", "msm_terms": n_total, "ntt_log_n": log_n,
                   "parallelism": f"range-shard x{world} + RCCL all-gather of partials" if world > 1 else "single GPU"},
        "roofline": {"bound": "hbm", "achieved": acc_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": acc_achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "msm_accumulate", "avg_ms": acc_avg_ms,
                     "note": "VALU int-MAD bound (see valu); algorithmic bytes = 128 B/term x terms per launch"},
        "ntt": {"metric": f"Fr NTT elements/sec @2^{log_n}", "value": world * n_ntt / ntt_s,
                "unit": "elements/s", "ms_per_ntt": ntt_s * 1e3, "scaling": "weak (one transform per GPU)",
                "ms_kernels_per_ntt": pass_ms / args.steps, "passes": passes_per_ntt,
                "roofline": {"bound": "hbm", "achieved": ntt_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": ntt_achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "ntt_pass",
                             "avg_ms": pass_avg_ms}},
        "checks": checks,
        "cpu_baseline": cpu_baseline,
    }
    print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
