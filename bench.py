#!/usr/bin/env python3
"""bench.py -- BLS12-381 G1 MSM point-adds/s @2^26 + Fr NTT elements/s @2^24 on MI355X.

Workload (BASELINE.json metric): one step = one G1 Pippenger MSM over 2^26
(base, scalar) terms.  The terms are sharded in contiguous ranges across the N
ranks (BASELINE config 4, multiexp.rs:332-336; at N=1 the whole 2^26 runs on
one GPU).  The per-rank partial sums are all-gathered over RCCL (linked into
libecgpu, ecg_msm_dist) and folded.  The host side of the launch (RCCL id,
barriers, max over ranks) runs over ecgpu.dist.HostGroup: this process never
imports torch, so the only HIP runtime and RCCL in it are the ROCm install's
(checked at start-up, ecg_runtime_info).

NTT legs: one in-place 2^24 Fr NTT per rank per step (radix_fft_many
semantics: whole transforms per GPU, no exchange; "ntt"), and at N > 1 one
2^24 NTT block-distributed over the N ranks (ecg_fft_dist, three RCCL
all-to-alls; "ntt_dist").

Inputs are synthetic and resident in HBM (library-owned device buffers)
before the timed region: bases P_i = (a + i*b) G generated on the GPU,
scalars uniform < r (seeded numpy, one stream per rank), NTT input uniform Fr.
value = total MSM terms / step time (whole job, max over ranks).

Checks, at every N, on rank 0 with the CPU oracle (the checker only):
the MSM result against the known answer (sum_j s_j (a + j b) mod r) G over all
2^26 terms (rank 0 regenerates every rank's scalars), the single-GPU NTT
bit-exactly against the CPU parallel_fft, and at N > 1 every rank's block of
the distributed NTT (SHA-256 digests) against the same parallel_fft.  Rank 0
at N=1 also times the CPU restatements as the baseline.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under
torch.distributed.run (one process per GPU), or plain `python bench.py --gpus N`,
which starts the N rank processes itself (launch_ranks) with the same
environment the launcher gives them.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402  (product path: libecgpu.so, fails loudly if missing)
from ecgpu import dist as edist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s
# v_mad_u64_u32 issue peak: 256 CUs x 4 SIMDs x 16 lanes per cycle (one wave64
# VALU instruction per 4 cycles per SIMD) at the 2.4 GHz peak clock
MAD_PEAK_T = 256 * 4 * 16 * 2.4e9 / 1e12
# measured int-MAD issue rate ("against a *measured* int-MAD peak"): a dependent-free
# stream of v_mad_u64_u32 issues one wave64 instruction per 4.5 SIMD cycles at 4 waves/SIMD
# (tools/issue_bench.hip, profiles/r02f/issue_bench.log), i.e. 256 x 4 x 64 / 4.5 per cycle
MAD_ISSUE_CYCLES = 4.5
MAD_PEAK_MEASURED_T = 256 * 4 * 64 / MAD_ISSUE_CYCLES * 2.4e9 / 1e12
R_BLS = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
R_BN = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
P_BLS = int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab", 16)
P_BN = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
MSM_SEED = 0x35A00026
NTT_SEED = 0x0FF70024
KAT_A = 0x1234567890ABCDEF1122334455667788
KAT_B = 0x0FEDCBA987654321
# reduced-radix limbs of the MSM's G1 Fq (fieldrr.hpp): 13 x 30 bits (BLS12-381, bls12_381_fq13_rr,
# split columns), 9 x 29 (BN254, bn254_fq9_rr); both tight-slack layouts (curve_rr.hpp)
RR_LIMBS = {0: 13, 1: 9}
RR_BITS = {0: 30, 1: 29}
# v_mad_u64_u32 per reduced-radix Fr product as ntt.hip executes it (9 x 29-bit limbs: 81 schoolbook +
# 81 reduction mads; BLS12-381's r = 1 mod 2^32 drops the m*P[0] mad of each of the 9 reduction columns
# in the ceil-carry form, fieldrr.hpp rr_ceil_carry)
FR_RR_MADS = {0: 2 * 9 * 9 - 9, 1: 2 * 9 * 9}


def madd_mads(nl: int) -> int:
    """v_mad_u64_u32 per XYZZ mixed add (rr_add_affine, curve_rr.hpp): three
    paired products (2 NL^2 each: schoolbook + Montgomery reduction) x 2, one
    paired squaring (NL(NL+1)/2 + NL^2) x 2, one product sum with a shared
    reduction (3 NL^2).  3055 for BLS12-381's 13 limbs (3542 with 14), 1467
    for BN254's 9 -- the main block's static count (tools/isa_count.py,
    profiles/r05/isa_accumulate_fq13.txt)."""
    mul, sqr = 2 * nl * nl, nl * (nl + 1) // 2 + nl * nl
    return 6 * mul + 2 * sqr + 3 * nl * nl


def ntt_fr_muls(log_n: int, max_deg: int = 10) -> float:
    """Fr products of one radix-2^d Stockham NTT as ntt.hip runs it: balanced
    passes of <= max_deg, radix-2^2 DIF steps (a quartet costs 1 + 3 (h-1)/h
    products: twiddles with qm = 0 are skipped), odd last round trivial, and
    one inter-pass twiddle per element with a non-zero exponent."""
    npass = -(-log_n // max_deg)
    degs = [log_n // npass + (1 if k < log_n % npass else 0) for k in range(npass)]
    n = 1 << log_n
    total, lgp = 0.0, 0
    for k, d in enumerate(degs):
        R = 1 << d
        r = 0
        while r + 1 < d:
            h = (R >> 2) >> r
            total += n / 4 * (1 + 3 * (h - 1) / h)
            r += 2
        if k > 0:
            total += n * (1 - 1 / (1 << lgp)) * (1 - 1 / R)
        lgp += d
    return total


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--msm-log", type=int, default=26)
    ap.add_argument("--ntt-log", type=int, default=24)
    ap.add_argument("--curve", default="bls12_381")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the oracle checks (profiling runs)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: EC_GPU_NUM_THREADS, else OMP_NUM_THREADS, else affinity)")
    ap.add_argument("--msm-cpu-log", type=int, default=24)
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive API timings (N=1)")
    ap.add_argument("--no-aux", action="store_true", help="skip the batched-MSM / EC-FFT side lines (N=1)")
    ap.add_argument("--no-table", action="store_true",
                    help="skip the window-table (fixed-base) MSM leg (ecg_msm_prepare_table)")
    ap.add_argument("--transport", choices=("rccl", "host"), default="rccl",
                    help="N > 1 exchange: RCCL over xGMI (one GPU per rank), or the host group "
                         "(ecg_comm_init_host over HostGroup: a rehearsal of the N > 1 path with several "
                         "ranks on one GPU, which RCCL refuses)")
    ap.add_argument("--single-device", action="store_true",
                    help="every rank on GPU 0 (with --transport host: N-rank rehearsal on a one-GPU box)")
    ap.add_argument("--msm-split", choices=("auto", "range", "grid"), default="auto",
                    help="N > 1 MSM split: 'range' = contiguous term shards (multiexp.rs:332-336, "
                         "ecg_msm_dist); 'grid' = every rank holds all bases and scalars and runs 1/N of the "
                         "(window x term) grid of the whole-n plan (ecg_msm_dist_grid, SURVEY §8(e)); 'auto' = "
                         "grid for BLS12-381 at N >= 4, where it measured faster per rank, else range "
                         "(DESIGN.md §7)")
    ap.add_argument("--unprepared", action="store_true",
                    help="time the MSM over [x, y] bases (conversion to the kernel layout inside every step)")
    return ap.parse_args(argv)


def cpu_threads(arg: int) -> int:
    """threadpool.rs:25-30: EC_GPU_NUM_THREADS, else every CPU this process may
    use (OMP_NUM_THREADS on the GPU box names its CPU share)."""
    if arg > 0:
        return arg
    for var in ("EC_GPU_NUM_THREADS", "OMP_NUM_THREADS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            return int(v)
    return len(os.sched_getaffinity(0))


def u64(x: int, n: int = 4) -> np.ndarray:
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)], dtype=np.uint64)


def rand_scalars(rng: np.random.Generator, n: int, r: int) -> np.ndarray:
    """uniform in [0, r) by rejection (vectorised)."""
    nbits = r.bit_length()
    out = np.empty((n, 4), dtype=np.uint64)
    top_mask = np.uint64((1 << (nbits - 192)) - 1)
    r_limbs = u64(r)
    filled = 0
    while filled < n:
        m = n - filled
        cand = rng.integers(0, 2**64, size=(m, 4), dtype=np.uint64)
        cand[:, 3] &= top_mask
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


def msm_shard(rank: int, world: int, n_total: int, r_int: int):
    """This rank's MSM shard: contiguous range (multiexp.rs:332-336), its
    scalars (seed stream [MSM_SEED, rank]) and the base generator offset:
    P_{i0 + i} = (KAT_A + (i0 + i) KAT_B) G = (a_loc + i KAT_B) G."""
    i0, i1 = edist.shard_range(n_total, world, rank)
    scal = rand_scalars(np.random.default_rng([MSM_SEED, rank]), i1 - i0, r_int)
    return i0, i1 - i0, scal, (KAT_A + i0 * KAT_B) % r_int


def msm_kat_scalar(co, cid: int, world: int, n_total: int, r_int: int, nthreads: int, shards=None) -> int:
    """sum_j s_j (KAT_A + j KAT_B) mod r over every rank's shard (regenerated
    from the per-rank seeds unless `shards` hands them in)."""
    k = 0
    for r in range(world):
        _, n_loc, scal, a_loc = shards[r] if shards is not None else msm_shard(r, world, n_total, r_int)
        if n_loc:
            k = (k + co.kat_scalar(cid, a_loc, KAT_B, scal, nthreads=nthreads)) % r_int
    return k


def omega_for(cid: int, r_int: int, ln: int) -> np.ndarray:
    """TWO_ADIC_ROOT^(2^(S - log n)) in Montgomery form (tests/fft.rs:16-24)."""
    gen, two_adicity = (7, 32) if cid == 0 else (5, 28)
    w = pow(gen, (r_int - 1) >> two_adicity, r_int)
    for _ in range(ln, two_adicity):
        w = w * w % r_int
    return u64(w * (1 << 256) % r_int)


def block_digests(a: np.ndarray, world: int) -> list:
    m = a.shape[0] // world
    return [hashlib.sha256(np.ascontiguousarray(a[r * m:(r + 1) * m]).tobytes()).hexdigest() for r in range(world)]


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv=None, grace_s: float = 60.0) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start the N rank
    processes here, one per GPU, with the environment torch.distributed.run
    gives them (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT), as the reference's MultiexpKernel spreads one
    multiexp over every device it holds (multiexp.rs:324-367, fft.rs:216-243).
    This parent never loads libecgpu or touches a GPU and never execs: the
    children inherit stdout / stderr (rank 0 alone prints the JSON line), and
    the exit code is the first failing rank's, after the others have been given
    `grace_s` to stop on their own (a failed rank fails every rank through the
    status records, comm.cpp) and are then killed."""
    import signal
    import subprocess

    argv = sys.argv[1:] if argv is None else list(argv)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(sys.argv[0]), *argv], env=env,
                                      start_new_session=True))
    rc, first_fail = 0, None
    t_start = t_beat = time.monotonic()
    try:
        while True:
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                break
            if time.monotonic() - t_beat > 30:  # a heartbeat: the ranks print only at the end
                t_beat = time.monotonic()
                print(f"bench: {sum(c is None for c in codes)} of {n} ranks running, "
                      f"{t_beat - t_start:.0f} s", file=sys.stderr, flush=True)
            failed = [c for c in codes if c not in (None, 0)]
            if failed and first_fail is None:
                first_fail = time.monotonic()
                rc = failed[0]
            if first_fail is not None and time.monotonic() - first_fail > grace_s:
                for p in procs:
                    if p.poll() is None:
                        os.killpg(p.pid, signal.SIGKILL)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        raise
    for r, p in enumerate(procs):
        if p.returncode != 0:
            print(f"bench: rank {r} of {n} exited with {p.returncode}", file=sys.stderr)
            rc = rc or p.returncode
    return 1 if rc and rc < 0 else rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)

    # the library (and through it the ROCm install's HIP runtime and RCCL) is
    # the first GPU code this process loads; torch is never imported
    runtime = ecgpu.lib().ecg_runtime_info().decode()
    if "/opt/rocm" not in runtime:
        raise SystemExit(f"libecgpu bound a foreign HIP runtime / RCCL: {runtime}")
    if rank == 0:
        print(f"runtime: {runtime}", file=sys.stderr)

    group = edist.HostGroup.from_env() if world > 1 else edist.HostGroup(0, 1)
    cid = ecgpu.CURVE_NAMES[args.curve]
    fr_fid = ecgpu.CURVE_FR_FIELD[cid]
    lq = ecgpu.CURVE_FQ_LIMBS[cid]
    r_int = R_BLS if cid == 0 else R_BN
    prog = ecgpu.program(ecgpu.Device(0 if args.single_device else local_rank))
    if world > 1 and args.transport == "host":
        edist.comm_init_host(prog, rank, world, edist.hostgroup_exchange(group))
    elif world > 1:
        edist.comm_init(prog, rank, world, group.broadcast)
    # what each rank's communicator itself reports (ranks, device PCI ids): rank 0's
    # record proves an N > 1 line ran N ranks on N distinct devices
    comm = edist.comm_record(group.allgather(edist.comm_info(prog))) if world > 1 else None
    nthreads = cpu_threads(args.cpu_threads)

    # ------------------------------------------------------------ MSM inputs (HBM-resident)
    n_total = 1 << args.msm_log
    split = args.msm_split
    if split == "auto":  # per-rank times on one GPU, profiles/r05/grid_split_probe_onecall_*.log
        split = "grid" if world >= 4 and cid == 0 else "range"
    grid = world > 1 and split == "grid"
    all_shards = None
    if grid:  # replicated operands: every rank holds all n_total bases and the scalars of every shard
        all_shards = [msm_shard(r, world, n_total, r_int) for r in range(world)]
        i0, n_loc, scal, a_loc = 0, n_total, np.concatenate([sh[2] for sh in all_shards]), KAT_A % r_int
    else:
        i0, n_loc, scal, a_loc = msm_shard(rank, world, n_total, r_int)
    d_scal = ecgpu.DeviceBuffer.upload(prog, scal)
    d_bases = ecgpu.gen_bases_dev(prog, args.curve, a_loc, KAT_B, n_loc)
    # upload_multiexp_bases (ag-cuda-ec/src/multiexp.rs:11-19): the resident
    # bases are held in the bucket kernels' own layout (128-B reduced-radix
    # records), converted once here -- as the reference uploads its bases once
    # and reuses them across multiexps.  --unprepared keeps the [x, y] layout
    # and converts inside every step.
    d_msm_bases = d_bases if args.unprepared else ecgpu.prepare_bases(prog, args.curve, d_bases, n_loc)
    result = np.zeros(3 * lq, dtype=np.uint64)

    def msm_step(bases=d_msm_bases):
        if world == 1:
            result[:] = ecgpu.msm_dev(prog, args.curve, bases, d_scal, n_loc)
        elif grid:  # 1/N of the (window x term) grid + the same [status | partial] all-gather + fold
            result[:] = edist.msm_dist_grid(prog, args.curve, bases, d_scal, n_total)
        else:  # local MSM + RCCL all-gather of world x 144 B partials + fold (no EC-add reduce op in RCCL)
            result[:] = edist.msm_dist(prog, args.curve, bases, d_scal, n_loc)

    # ------------------------------------------------------------ NTT inputs (HBM-resident)
    log_n = args.ntt_log
    n_ntt = 1 << log_n
    omega_m = omega_for(cid, r_int, log_n)
    # any value < r is a Montgomery form; every rank holds the same seeded input
    ntt_in = rand_scalars(np.random.default_rng([NTT_SEED, 0]), n_ntt, r_int)
    d_ntt = ecgpu.DeviceBuffer.upload(prog, ntt_in)

    def ntt_step():
        # in place; back-to-back steps transform the previous output (still uniform Fr data)
        ecgpu.fft_dev(prog, args.curve + "_fr", d_ntt, omega_m, log_n)

    def barrier():
        # every libecgpu call returns after its stream is synchronised, so the
        # device is idle here; the barrier lines the ranks up
        prog.synchronize()
        group.barrier()

    # ------------------------------------------------------------ MSM timing (every call is synchronous)
    for _ in range(args.warmup):
        msm_step()
    barrier()
    t0 = time.perf_counter()
    acc_ms = 0.0
    acc_launch = 0
    for _ in range(args.steps):
        msm_step()
        ms, cnt = prog.kernel_time("msm_accumulate")
        acc_ms += ms
        acc_launch += cnt
    barrier()
    msm_s = group.max(time.perf_counter() - t0) / args.steps
    acc_avg_ms = group.max(acc_ms / max(acc_launch, 1))
    if grid:  # up to three pieces of different sizes per step: the roofline takes the per-step sum
        acc_avg_ms = group.max(acc_ms / args.steps)
    if comm is not None:  # the last step's status + partial all-gather, slowest rank
        comm["msm_allgather_us"] = group.max(edist.last_exchange_us(prog))
    msm_result = result.copy()
    # the same MSM over the [x, y] bases, converting them inside the step (reported, not `value`)
    unprep_ms = None
    if not args.unprepared:
        msm_step(d_bases)
        barrier()
        t0 = time.perf_counter()
        for _ in range(2):
            msm_step(d_bases)
        barrier()
        unprep_ms = group.max(time.perf_counter() - t0) / 2 * 1e3
        if not (result == msm_result).all():  # every rank holds the folded result
            raise SystemExit("prepared and unprepared MSM results differ")

    # the same MSM over a window table of the bases (fixed-base form, ecg_msm_prepare_table): reported
    # beside `value`, which stays on the per-call base layout the reference's API takes
    table = None
    if not args.no_table and not args.unprepared and cid in (0, 1) and not grid:
        msm_prep = d_msm_bases
        t0 = time.perf_counter()
        d_tab = ecgpu.prepare_bases(prog, args.curve, d_bases, n_loc, window_table=0)
        prep_s = group.max(time.perf_counter() - t0)
        msm_step(d_tab)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            msm_step(d_tab)
        barrier()
        tab_s = group.max(time.perf_counter() - t0) / args.steps
        table = {"ms": tab_s * 1e3, "value": n_total / tab_s, "unit": "point-adds/s",
                 "window": ecgpu.lib().ecg_msm_table_window(cid, n_loc), "prepare_s": prep_s,
                 "equals_headline_result": bool((result == msm_result).all()),
                 "note": "bases prepared with their 2^(k c) multiples (W rows): every window feeds one bucket set; "
                         "same inputs and result as `value`, table built once outside the timed region"}
        d_tab.free()
        del msm_prep

    # ------------------------------------------------------------ NTT timing (one transform per GPU)
    for _ in range(args.warmup):
        ntt_step()
    barrier()
    t0 = time.perf_counter()
    pass_ms, pass_launch = 0.0, 0
    for _ in range(args.steps):
        ntt_step()
        ms, cnt = prog.kernel_time("ntt_pass")
        pass_ms += ms
        pass_launch += cnt
    barrier()
    ntt_s = group.max(time.perf_counter() - t0) / args.steps
    pass_avg_ms = group.max(pass_ms / max(pass_launch, 1))
    passes_per_ntt = pass_launch / args.steps

    # ------------------------------------------------------------ distributed NTT (N > 1): one 2^24 over all ranks
    ntt_dist = None
    dist_digests = None
    if world > 1:
        m = n_ntt // world
        d_blk = ecgpu.DeviceBuffer.upload(prog, ntt_in[rank * m:(rank + 1) * m])
        for _ in range(args.warmup):
            edist.fft_dist(prog, args.curve + "_fr", d_blk, omega_m, log_n)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            edist.fft_dist(prog, args.curve + "_fr", d_blk, omega_m, log_n)
        barrier()
        fd_s = group.max(time.perf_counter() - t0) / args.steps
        # checked run: fresh input block, one transform
        d_blk.write(ntt_in[rank * m:(rank + 1) * m])
        edist.fft_dist(prog, args.curve + "_fr", d_blk, omega_m, log_n)
        blk = d_blk.read(shape=(m, 4))
        dist_digests = group.allgather(hashlib.sha256(blk.tobytes()).hexdigest())
        d_blk.free()
        ntt_dist = {"metric": f"Fr NTT elements/sec @2^{log_n}, one transform block-distributed over {world} GPUs",
                    "value": n_ntt / fd_s, "unit": "elements/s", "ms_per_ntt": fd_s * 1e3, "scaling": "strong",
                    "exchange": "3 RCCL all-to-alls of 32*m*(N-1)/N B per rank (dfft.hip)"}

    # ------------------------------------------------------------ oracle leg (rank 0): checks + CPU baseline
    # The CPU oracle (oracle/) is used only here: as the checker and as the
    # timed CPU baseline, never on the measured path.
    checks = {}
    cpu_baseline = None
    if rank == 0 and not args.no_check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle as co

        # MSM known answer over all 2^26 terms (SURVEY §8c KAT), every rank's shard
        shards = [(i0, n_loc, scal, a_loc)] if world == 1 else all_shards
        kat = msm_kat_scalar(co, cid, world, n_total, r_int, nthreads, shards)
        want = co.jac_to_affine(cid, co.gen_mul(cid, kat))
        got = co.jac_to_affine(cid, msm_result)
        checks[f"msm_kat_2^{args.msm_log}"] = bool(want is not None and got is not None and (want == got).all())
        # NTT: fresh transform of the seeded input vs CPU parallel_fft (fft_cpu.rs:59-111), bit-exact
        d_ntt.write(ntt_in)
        ntt_step()
        gpu_out = d_ntt.read(shape=(n_ntt, 4))
        lt = max(0, min(log_n - 1, nthreads.bit_length() - 1))  # worker.log_num_threads()
        t_cpu = time.perf_counter()
        ref = co.parallel_fft(fr_fid, ntt_in, omega_m, log_n, lt)
        ntt_cpu_s = time.perf_counter() - t_cpu
        print(f"CPU ({1 << lt} cores) took {ntt_cpu_s * 1e3:.0f}ms", file=sys.stderr)  # tests/fft.rs:77
        checks[f"ntt_vs_parallel_fft_2^{log_n}"] = bool((gpu_out == ref).all())
        if dist_digests is not None:
            checks[f"ntt_dist_{world}gpu_vs_parallel_fft_2^{log_n}"] = dist_digests == block_digests(ref, world)
        if world == 1 and not args.no_cpu_baseline:
            # CPU baseline: multiexp_cpu restatement on a bounded sample of the same workload
            ns = min(1 << args.msm_cpu_log, n_loc)
            sb = np.ascontiguousarray(d_bases.read(shape=(n_loc, 2 * lq))[:ns])
            ss = np.ascontiguousarray(scal[:ns])
            t_cpu = time.perf_counter()
            co.multiexp_cpu(cid, sb, ss, nthreads=nthreads)
            cpu_s = time.perf_counter() - t_cpu
            print(f"CPU ({nthreads} cores) took {cpu_s * 1e3:.0f}ms (multiexp_cpu, {ns} terms)", file=sys.stderr)
            del sb
            cpu_baseline = {
                "value": ns / cpu_s, "unit": "point-adds/s", "cores": nthreads, "kind": "port",
                "sample": f"multiexp_cpu restatement (oracle/oracle.c; c=ceil(ln N), windows in parallel) on the "
                          f"first 2^{ns.bit_length() - 1} terms of the same inputs: {cpu_s:.2f} s wall",
                "ntt": {"value": n_ntt / ntt_cpu_s, "unit": "elements/s", "cores": 1 << lt, "kind": "port",
                        "sample": f"parallel_fft restatement at the full 2^{log_n}: {ntt_cpu_s:.2f} s wall"},
            }

    # ------------------------------------------------------------ end-to-end API (PCIe-inclusive), N = 1
    # The reference API takes host slices and copies them in and out on every
    # call (multiexp.rs:163-164, fft.rs:89,129).  Not `value`: DESIGN.md §6.
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        host_bases = d_bases.read(shape=(n_loc, 2 * lq))
        kern = ecgpu.MultiexpKernel.create([prog], [], args.curve)
        pool = ecgpu.Worker()
        kern.multiexp(pool, host_bases, scal, 0)
        t_e = time.perf_counter()
        out_e2e = kern.multiexp(pool, host_bases, scal, 0)
        msm_e2e_s = time.perf_counter() - t_e
        checks["msm_e2e_equals_resident"] = bool((out_e2e == msm_result).all())
        # as the Rust drop-in calls it (MultiexpKernel::multiexp(pool, Arc<Vec<Affine>>, exps, skip)):
        # arkworks Affine {x, y, infinity} records straight from the caller, converted on the device and
        # kept resident in the base cache; the first call uploads and prepares them, the second with the
        # same array uploads only the exponents (pipelined with the compute)
        ark = np.zeros((n_loc, 2 * lq + 1), dtype=np.uint64)
        ark[:, :2 * lq] = host_bases
        del host_bases
        kern.clear_base_cache()
        t_e = time.perf_counter()
        out_cold = kern.multiexp_ex(ark, scal, 0, ark_affine=True, cache_bases=True)
        ark_cold_s = time.perf_counter() - t_e
        ark_cached = []
        for _ in range(3):
            t_e = time.perf_counter()
            out_warm = kern.multiexp_ex(ark, scal, 0, ark_affine=True, cache_bases=True)
            ark_cached.append(time.perf_counter() - t_e)
        checks["msm_ark_cached_equals_resident"] = bool((out_cold == msm_result).all()
                                                        and (out_warm == msm_result).all())
        kern.clear_base_cache()
        del ark
        host_bases = None
        fk = ecgpu.FftKernel.create([prog], args.curve + "_fr")
        host_ntt = ntt_in.copy()
        fk.radix_fft(host_ntt, omega_m, log_n)
        host_ntt = ntt_in.copy()
        t_e = time.perf_counter()
        fk.radix_fft(host_ntt, omega_m, log_n)
        ntt_e2e_s = time.perf_counter() - t_e
        e2e = {"msm_ms": msm_e2e_s * 1e3, "msm_terms_per_s": n_loc / msm_e2e_s,
               "msm_ark_cold_ms": ark_cold_s * 1e3, "msm_ark_cached_ms": min(ark_cached) * 1e3,
               "msm_ark_cached_ms_all": [t * 1e3 for t in ark_cached],
               "ntt_ms": ntt_e2e_s * 1e3, "ntt_elements_per_s": n_ntt / ntt_e2e_s,
               "note": "host buffers in, host result out. msm_ms: GpuRepr [x, y] slices (ecg_msm, H2D of 128 B/term "
                       "pipelined with compute); msm_ark_*: arkworks Affine records (104 B/base) as the Rust "
                       "MultiexpKernel::multiexp passes its Arc<Vec<G>> (ecg_msm_ex, ark layout, base cache): "
                       "cold = upload + device conversion + prepare + MSM, cached = the same Arc again (only the "
                       "32-B exponents travel, in passes behind the compute); NTT: H2D+D2H of 32 B/element"}

    # ------------------------------------------------------------ side lines (N = 1): SURVEY §8f rows
    aux = None
    if rank == 0 and world == 1 and not args.no_aux:
        aux = {}
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle as co20  # checker only (KAT / inputs), never timed
        # BASELINE config 3: G1 MSM at 2^20 -- the first 2^20 resident terms, KAT-checked
        n20 = 1 << 20
        if n_loc >= n20:
            ecgpu.msm_dev(prog, args.curve, d_msm_bases, d_scal, n20)
            best20 = 1e9
            for _ in range(5):
                t_a = time.perf_counter()
                out20 = ecgpu.msm_dev(prog, args.curve, d_msm_bases, d_scal, n20)
                best20 = min(best20, time.perf_counter() - t_a)
            k20 = co20.kat_scalar(cid, a_loc, KAT_B, scal[:n20], nthreads=nthreads) % r_int
            want20 = co20.jac_to_affine(cid, co20.gen_mul(cid, k20))
            got20 = co20.jac_to_affine(cid, out20)
            aux["msm_2p20"] = {"ms": best20 * 1e3, "point_adds_per_s": n20 / best20,
                               "kat": bool(want20 is not None and got20 is not None and (want20 == got20).all()),
                               "note": "BASELINE config 3: first 2^20 resident terms, best of 5 synchronous calls"}
        # the reference's own multiexp bench (ag-cuda-ec/benches/multiexp.rs:15-62): 2^22 bases cycled
        # with period 99, scalars with period 73, multiple_multiexp_st(.., 1024 chunks, window 8, false)
        nrb = 1 << 22
        meta_b = co20.gen_bases(cid, 41, 43, 99)
        d_rb = ecgpu.upload_multiexp_bases(prog, np.ascontiguousarray(np.resize(meta_b, (nrb, meta_b.shape[1]))),
                                           curve=args.curve)
        meta_e = rand_scalars(np.random.default_rng(73), 73, r_int)
        d_re = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(np.resize(meta_e, (nrb, 4))))
        out_rb = ecgpu.multiple_multiexp(prog, d_rb, (d_re, nrb), 1024, 8, False, curve=args.curve)
        best_rb = 1e9
        for _ in range(3):
            t_a = time.perf_counter()
            ecgpu.multiple_multiexp(prog, d_rb, (d_re, nrb), 1024, 8, False, curve=args.curve)
            best_rb = min(best_rb, time.perf_counter() - t_a)
        aux["reference_multiexp_bench_shape"] = {
            "shape": "2^22 terms (bases period 99, scalars period 73), 1024 tasks of 4096, window 8",
            "ms": best_rb * 1e3, "terms_per_s": nrb / best_rb,
            "note": "the reference prints this as 'GPU took {}ms' (bases already uploaded here)"}
        d_rb.free()
        if not args.no_table and cid in (0, 1):
            # the same call over bases uploaded in the window-table form -- the Rust
            # upload_multiexp_bases_table(bases, 4096, 0) path (ecg_msm_prepare_table, one bucket set per task)
            tw_r = ecgpu.lib().ecg_msm_table_window(cid, nrb // 1024)
            t_a = time.perf_counter()
            d_rt = ecgpu.upload_multiexp_bases(prog, np.ascontiguousarray(np.resize(meta_b, (nrb, meta_b.shape[1]))),
                                               curve=args.curve, window_table=tw_r)
            rt_prep = time.perf_counter() - t_a
            out_rt = ecgpu.multiple_multiexp(prog, d_rt, (d_re, nrb), 1024, 8, False, curve=args.curve)
            best_rt = 1e9
            for _ in range(3):
                t_a = time.perf_counter()
                ecgpu.multiple_multiexp(prog, d_rt, (d_re, nrb), 1024, 8, False, curve=args.curve)
                best_rt = min(best_rt, time.perf_counter() - t_a)
            aux["reference_multiexp_bench_shape_table"] = {
                "window": tw_r, "upload_and_prepare_s": rt_prep, "ms": best_rt * 1e3, "terms_per_s": nrb / best_rt,
                "equal": bool((out_rt == out_rb).all()),
                "note": "bases uploaded once with their window table (upload_multiexp_bases_table)"}
            d_rt.free()
        d_re.free()
        # batched multi-line MSM on the ag-cuda-ec AMT shape (benches/amt.rs: LOG_N=10 -> 2^21 x 10 lines)
        L, lines, chunks = 1 << 21, 10, 1 << 10
        d_lb = ecgpu.gen_bases_dev(prog, args.curve, 7, 11, L * lines)
        d_le = ecgpu.DeviceBuffer.upload(prog, rand_scalars(np.random.default_rng(5), L, r_int))
        ecgpu.multiple_multiexp(prog, d_lb, (d_le, L), chunks, curve=args.curve)
        t_a = time.perf_counter()
        ecgpu.multiple_multiexp(prog, d_lb, (d_le, L), chunks, curve=args.curve)
        mm_s = time.perf_counter() - t_a
        aux["multiple_multiexp"] = {"shape": f"{lines} lines x 2^21, {chunks} chunks/line ({L // chunks} terms/task)",
                                    "ms": mm_s * 1e3, "terms_per_s": L * lines / mm_s}
        if not args.no_table and cid in (0, 1):
            # the AMT bases are uploaded once and reused (upload_multiexp_bases): window table for 2^11-term tasks
            mm_ref = ecgpu.multiple_multiexp(prog, d_lb, (d_le, L), chunks, curve=args.curve)
            tw = ecgpu.lib().ecg_msm_table_window(cid, L // chunks)
            t_a = time.perf_counter()
            d_lt = ecgpu.prepare_bases(prog, args.curve, d_lb, L * lines, window_table=tw)
            lt_prep = time.perf_counter() - t_a
            ecgpu.multiple_multiexp(prog, d_lt, (d_le, L), chunks, curve=args.curve)
            t_a = time.perf_counter()
            mm_t = ecgpu.multiple_multiexp(prog, d_lt, (d_le, L), chunks, curve=args.curve)
            mt_s = time.perf_counter() - t_a
            aux["multiple_multiexp_window_table"] = {"window": tw, "prepare_s": lt_prep, "ms": mt_s * 1e3,
                                                     "terms_per_s": L * lines / mt_s,
                                                     "equal": bool((mm_t == mm_ref).all())}
            d_lt.free()
        d_lb.free()
        d_le.free()
        # G1 EC-FFT 2^16 (tests/ec_fft.rs top size)
        le = 16
        d_pts = ecgpu.gen_bases_dev(prog, args.curve, 3, 7, 1 << le)
        aff = d_pts.read(shape=(1 << le, 2 * lq))
        one = u64(((1 << (64 * lq)) % (P_BLS if cid == 0 else P_BN)), lq)
        jac = np.ascontiguousarray(np.concatenate([aff, np.tile(one, (1 << le, 1))], axis=1))
        d_jac = ecgpu.DeviceBuffer.upload(prog, jac)
        om_e = omega_for(cid, r_int, le)
        ecgpu.ec_fft_dev(prog, args.curve, d_jac, om_e, le)
        d_jac.write(jac)
        t_a = time.perf_counter()
        ecgpu.ec_fft_dev(prog, args.curve, d_jac, om_e, le)
        ef_s = time.perf_counter() - t_a
        aux["ec_fft"] = {"log_n": le, "ms": ef_s * 1e3, "butterflies_per_s": (1 << (le - 1)) * le / ef_s}
        # the smaller sizes 0g runs (2^10-2^14): point operations on lane quads / pairs
        small = {}
        for ls in (10, 12, 14):
            ns = 1 << ls
            d_s = ecgpu.DeviceBuffer.upload(prog, np.ascontiguousarray(jac[:ns]))
            om_s = omega_for(cid, r_int, ls)
            ecgpu.ec_fft_dev(prog, args.curve, d_s, om_s, ls)
            d_s.write(np.ascontiguousarray(jac[:ns]))
            t_a = time.perf_counter()
            ecgpu.ec_fft_dev(prog, args.curve, d_s, om_s, ls)
            small[str(ls)] = (time.perf_counter() - t_a) * 1e3
            d_s.free()
        aux["ec_fft_small_ms"] = small
        # the reference's own EC-FFT bench (ag-cuda-ec/benches/ec_fft.rs:20-55): degrees 0..11, one
        # radix_ec_fft_st call each on host points (its "GPU took {}ms" includes the copies in and out)
        ek1 = ecgpu.EcFftKernel.create([prog], args.curve)
        seq = {}
        for deg in range(0, 12):
            x = np.ascontiguousarray(jac[:1 << deg])
            om_d = omega_for(cid, r_int, deg)
            ek1.radix_ec_fft(x.copy(), om_d, deg)  # first call of a size builds its twiddles
            best = 1e9
            for _ in range(3):
                y = x.copy()
                t_a = time.perf_counter()
                ek1.radix_ec_fft(y, om_d, deg)
                best = min(best, time.perf_counter() - t_a)
            seq[str(deg)] = best * 1e3
        aux["reference_ec_fft_bench_sequential_ms"] = {
            "ms_by_log_n": seq,
            "note": "benches/ec_fft.rs bench_ec_fft_sequential: one radix_ec_fft per degree 0..11, host points in and "
                    "out, best of 3 after one warm call"}
        # benches/ec_fft.rs:62-112 bench_ec_fft_parallel: 32 concurrent tasks, each a forward and an
        # inverse 2^6 transform on its own thread-local workspace (here: 32 threads, one context each)
        import threading
        ln6, tasks = 6, 32
        om6 = omega_for(cid, r_int, ln6)
        om6_inv = u64(pow(int(sum(int(v) << (64 * i) for i, v in enumerate(om6))) * pow(1 << 256, -1, r_int)
                          % r_int, -1, r_int) * (1 << 256) % r_int)
        tprogs = [ecgpu.program(ecgpu.Device(0 if args.single_device else local_rank)) for _ in range(tasks)]
        tks = [ecgpu.EcFftKernel.create([tp], args.curve) for tp in tprogs]
        xs6 = [np.ascontiguousarray(jac[(i << ln6):((i + 1) << ln6)]) for i in range(tasks)]

        def par_round():
            ys = [x.copy() for x in xs6]

            def task(i):
                tks[i].radix_ec_fft(ys[i], om6, ln6)
                tks[i].radix_ec_fft(ys[i], om6_inv, ln6)

            th = [threading.Thread(target=task, args=(i,)) for i in range(tasks)]
            t_a = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            return time.perf_counter() - t_a, ys

        par_round()
        par_s, ys6 = min((par_round() for _ in range(3)), key=lambda v: v[0])
        # forward then inverse = n x the input (the bench's own check, ec_fft.rs:104-108)
        scale_ok = True
        n6 = co20.u64arr([1 << ln6], 4)
        for i in (0, tasks - 1):
            want6 = [co20.jac_to_affine(cid, co20.naive_multiexp(cid, np.ascontiguousarray(xs6[i][j:j + 1, :2 * lq]),
                                                                 n6)) for j in range(1 << ln6)]
            got6 = [co20.jac_to_affine(cid, ys6[i][j]) for j in range(1 << ln6)]
            scale_ok = scale_ok and all((a is None and b is None) or (a is not None and b is not None and (a == b).all())
                                        for a, b in zip(want6, got6))
        for tp in tprogs:
            tp.close()
        aux["reference_ec_fft_bench_parallel"] = {
            "tasks": tasks, "log_n": ln6, "ms": par_s * 1e3, "ms_per_task_pair": par_s * 1e3 / tasks,
            "forward_inverse_is_n_times_input": bool(scale_ok),
            "note": "benches/ec_fft.rs bench_ec_fft_parallel: 32 threads, each forward + inverse 2^6 on its own "
                    "context, host points; wall time of the whole set, best of 3"}
        d_jac.free()
        d_pts.free()
        # radix_ec_fft_many over 16 same-size inputs (the 2^16 points cut into 2^12
        # slices): one batched transform, beside one radix_ec_fft call per input
        lm, cm = 12, 16
        ek = ecgpu.EcFftKernel.create([prog], args.curve)
        om_m = omega_for(cid, r_int, lm)
        xs = [np.ascontiguousarray(jac[i << lm:(i + 1) << lm]) for i in range(cm)]
        ys = [x.copy() for x in xs]
        t_a = time.perf_counter()
        ek.radix_ec_fft_many(xs, [om_m] * cm, [lm] * cm)
        em_s = time.perf_counter() - t_a
        t_a = time.perf_counter()
        for y in ys:
            ek.radix_ec_fft(y, om_m, lm)
        e1_s = time.perf_counter() - t_a
        aux["ec_fft_many"] = {"log_n": lm, "count": cm, "ms": em_s * 1e3, "ms_one_call_per_input": e1_s * 1e3,
                              "equal": all(bool((x == y).all()) for x, y in zip(xs, ys)),
                              "note": "host buffers in and out (EcFftKernel::radix_ec_fft_many); the run of "
                                      "equal-size, equal-omega inputs is one batched transform"}
        # G2 MSM over Fq2: 2^22 terms, prepared bases, KAT-checked
        g2 = args.curve + "_g2"
        lg = 22
        ng = 1 << lg
        d_gb = ecgpu.gen_bases_dev(prog, g2, KAT_A % r_int, KAT_B, ng)
        d_gp = ecgpu.prepare_bases(prog, g2, d_gb, ng)
        d_gb.free()
        gs = rand_scalars(np.random.default_rng([MSM_SEED, 22]), ng, r_int)
        d_gs = ecgpu.DeviceBuffer.upload(prog, gs)
        out_g2 = ecgpu.msm_dev(prog, g2, d_gp, d_gs, ng)
        t_a = time.perf_counter()
        for _ in range(2):
            out_g2 = ecgpu.msm_dev(prog, g2, d_gp, d_gs, ng)
        g2_s = (time.perf_counter() - t_a) / 2
        aux["g2_msm"] = {"log_n": lg, "ms": g2_s * 1e3, "point_adds_per_s": ng / g2_s,
                         "kat": bool(_g2_kat(cid, gs, r_int, out_g2))}
        d_gp.free()
        d_gs.free()
        # G2 EC-FFT 2^12 (component-split lane pairs): device-resident Jacobian points
        l2 = 12
        lq2 = 2 * lq
        aff2 = ecgpu.gen_bases_dev(prog, g2, 3, 7, 1 << l2).read(shape=(1 << l2, 2 * lq2))
        one2 = np.zeros(lq2, dtype=np.uint64)
        one2[:lq] = one
        jac2 = np.ascontiguousarray(np.concatenate([aff2, np.tile(one2, (1 << l2, 1))], axis=1))
        d_j2 = ecgpu.DeviceBuffer.upload(prog, jac2)
        om_2 = omega_for(cid, r_int, l2)
        ecgpu.ec_fft_dev(prog, g2, d_j2, om_2, l2)
        d_j2.write(jac2)
        t_a = time.perf_counter()
        ecgpu.ec_fft_dev(prog, g2, d_j2, om_2, l2)
        aux["g2_ec_fft"] = {"log_n": l2, "ms": (time.perf_counter() - t_a) * 1e3}
        d_j2.free()
        # the reference's ag-cuda-ec benches with their own checks, on this curve and (default
        # run) on BN254, the curve those benches compile for (ag-cuda-ec/Cargo.toml:36)
        dev_index = 0 if args.single_device else local_rank
        for key, cv in (("reference_benches", args.curve),) + ((("reference_benches_bn254", "bn254"),) if cid == 0 else ()):
            try:
                aux[key] = reference_bench_suite(prog, cv, dev_index, nthreads, co20)
            except Exception as e:  # a side line must not sink the headline line
                aux[key] = {"error": f"{type(e).__name__}: {e}"}

    if rank != 0:
        group.barrier()
        group.close()
        return

    # ------------------------------------------------------------ report
    # terms per accumulation launch on rank 0 (the largest shard); grid split:
    # a rank's W n / N grid cells per step count as n / N terms of W windows
    n_acc = n_total // world if grid else n_loc
    W = -(-(r_int.bit_length() + 1) // 20) if args.msm_log >= 24 else None  # windows at c = 20
    bytes_per_term = 2 * lq * 8 + 32  # affine + 32 B scalar: 128 B (BLS12-381), 96 B (BN254), SURVEY §8(d)
    hbm_achieved = bytes_per_term * n_acc / (acc_avg_ms / 1e3) / 1e9
    # the committed PMC passes profile the default (BLS12-381, 2^26 / 2^24) run
    default_run = cid == 0 and args.msm_log == 26 and log_n == 24 and world == 1
    acc_traffic, acc_src = pmc_traffic("msm_accumulate") if default_run else (None, None)
    ntt_traffic, ntt_src = pmc_traffic("ntt_pass") if default_run else (None, None)
    if cid == 1 and world == 1:  # BN254 (config 5): its own committed PMC passes
        bn = os.path.join(ROOT, "profiles", "pmc_bn254_current.json")
        try:
            with open(bn) as f:
                d_bn = json.load(f)
            if args.msm_log == 26:
                acc_traffic, acc_src = d_bn["traffic_gb_per_launch"], d_bn["source"]
            if log_n == 24 and "ntt_traffic_gb_per_launch" in d_bn:
                ntt_traffic, ntt_src = d_bn["ntt_traffic_gb_per_launch"], d_bn["ntt_source"]
        except (OSError, ValueError, KeyError, TypeError) as e:
            print(f"bench: ignoring {bn}: {type(e).__name__}: {e}", file=sys.stderr)
    ntt_achieved = 64 * n_ntt / (pass_avg_ms / 1e3) / 1e9
    roofline = {"bound": "valu", "kernel": "msm_accumulate", "avg_ms": acc_avg_ms,
                "traffic": acc_traffic, "traffic_unit": "GB/launch", "traffic_source": acc_src}
    if W and cid in RR_LIMBS:
        mads = madd_mads(RR_LIMBS[cid])
        achieved = n_acc * W * mads / (acc_avg_ms / 1e3) / 1e12
        roofline.update({"achieved": achieved, "peak": MAD_PEAK_T, "unit": "T v_mad_u64_u32/s",
                         "frac": achieved / MAD_PEAK_T,
                         "measured_peak": {"peak": MAD_PEAK_MEASURED_T, "frac": achieved / MAD_PEAK_MEASURED_T,
                                           "note": f"{MAD_ISSUE_CYCLES} SIMD cycles per wave64 v_mad_u64_u32 "
                                                   "(tools/issue_bench.hip) at 2.4 GHz"},
                         "mads_per_add": mads, "mixed_adds_per_s": n_acc * W / (acc_avg_ms / 1e3),
                         "note": f"{mads} v_mad_u64_u32 per XYZZ mixed add (8M+2S, {RR_LIMBS[cid]} x {RR_BITS[cid]}-bit limbs"
                                 + ("; BLS12-381's 13 x 30-bit layout issues 14 % fewer mads per add than round 4's "
                                    "14 x 29 bits, so this fraction is lower while mixed_adds_per_s is higher" if cid == 0
                                    else "; BN254's tight-slack 9 x 29-bit layout: 2117 VALU per add, 1467 of them mads")
                                 + f") x {W} windows x terms / launch time; peak = 256 CU x 4 SIMD x 16 lanes x 2.4 GHz"})
    roofline["hbm"] = {"achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": hbm_achieved / HBM_PEAK_GBS,
                       "note": f"algorithmic {bytes_per_term} B/term ({2 * lq * 8} B base + 32 B scalar) x terms "
                               "per launch / launch time"}
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
        "dtype": ("mod-p integer on v_mad_u64_u32 (reduced-radix Montgomery: MSM Fq "
                  + f"{RR_LIMBS[cid]} x {RR_BITS[cid]}-bit" + " limbs, NTT Fr 9 x 29-bit)"),
        "data": "synthetic: bases (a+i*b)G generated on GPU, scalars uniform < r (seeded), HBM-resident"
                + ("" if args.unprepared else "; bases prepared once in the kernels' 128-B record layout "
                   "(ecg_msm_prepare_bases, upload_multiexp_bases's role)"),
        "config": {"workload": f"{args.curve} G1 MSM 2^{args.msm_log} terms sharded over {world} GPU(s) "
                               f"+ Fr NTT 2^{log_n} per GPU", "msm_terms": n_total, "ntt_log_n": log_n,
                   "msm_split": split if world > 1 else None,
                   "parallelism": ((f"grid split (window x term) x{world}, replicated bases + " if grid
                                    else f"range-shard x{world} + ")
                                   + ("RCCL" if args.transport == "rccl" else "host-group (rehearsal)")
                                   + " all-gather of partials") if world > 1 else "single GPU"},
        "msm_ms_unprepared_bases": unprep_ms,
        "msm_window_table": table,
        "roofline": roofline,
        "ntt": {"metric": f"Fr NTT elements/sec @2^{log_n}", "value": world * n_ntt / ntt_s,
                "unit": "elements/s", "ms_per_ntt": ntt_s * 1e3, "scaling": "weak (one transform per GPU)",
                "ms_kernels_per_ntt": pass_ms / args.steps, "passes": passes_per_ntt,
                "roofline": {"bound": "valu", "achieved": ntt_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": ntt_achieved / HBM_PEAK_GBS, "traffic": ntt_traffic,
                             "traffic_unit": "GB/launch", "traffic_source": ntt_src, "kernel": "ntt_pass",
                             "avg_ms": pass_avg_ms, "note": "HBM fraction of a VALU-bound pass (64 B/element)"}},
        "ntt_dist": ntt_dist,
        "rccl": comm,
        "checks": checks,
        "cpu_baseline": cpu_baseline,
        "e2e_api": e2e,
        "aux": aux,
        "runtime": runtime,
    }
    muls = ntt_fr_muls(log_n)
    # reduced-radix Fr product (fieldrr.hpp, 9 x 29-bit limbs): 81 schoolbook + 81 reduction mads
    mad_rate = muls * FR_RR_MADS[cid] / (pass_ms / args.steps / 1e3) / 1e12
    line["ntt"]["valu"] = {"kernel": "ntt_pass", "achieved": mad_rate, "peak": MAD_PEAK_T,
                           "unit": "T v_mad_u64_u32/s", "frac": mad_rate / MAD_PEAK_T,
                           "note": f"{muls / n_ntt:.2f} Fr products per element per transform x {FR_RR_MADS[cid]} "
                                   "v_mad_u64_u32 / kernel time; peak as the MSM roofline's"}
    print(json.dumps(line))
    group.barrier()
    group.close()


def _fold_points(co, cid: int, pts: np.ndarray) -> np.ndarray:
    """sum of normalised Jacobian points on the host (checker only)."""
    lq = ecgpu.CURVE_FQ_LIMBS[cid]
    acc = np.zeros(3 * lq, dtype=np.uint64)
    for p in np.asarray(pts, dtype=np.uint64).reshape(-1, 3 * lq):
        co.lib().orc_jac_add(cid, co.ptr(acc), co.ptr(acc), co.ptr(np.ascontiguousarray(p)))
    return acc


def _same_point(co, cid: int, a: np.ndarray, b: np.ndarray) -> bool:
    x, y = co.jac_to_affine(cid, a), co.jac_to_affine(cid, b)
    return (x is None and y is None) or (x is not None and y is not None and bool((x == y).all()))


def reference_bench_suite(prog, curve: str, dev_index: int, nthreads: int, co) -> dict:
    """The reference's own ag-cuda-ec benches on `curve`, each with the check
    the bench itself makes (ag-cuda-ec compiles them for BN254 by default,
    Cargo.toml:36 + pairing_suite.rs:1-12):
      * benches/multiexp.rs:15-62: 2^22 terms (bases cycled with period 99,
        scalars with period 73), multiple_multiexp_st(.., 1024, 8, false);
        check: the sum of the 1024 task results == the CPU MSM of all terms;
      * benches/amt.rs:14-56: 10 lines of 2^21 bases (period 97), one row of
        2^21 scalars (period 73), group degrees 7..11 with the engine's own
        window, then the bench's whole grid (group degree 7..11 x window size
        4..9, the window pinned); check: every run's task results sum to the
        same per-line points, and line 0 equals the CPU MSM;
      * benches/ec_fft.rs:20-55: one radix_ec_fft per degree 0..11 on host
        points, checked against serial_ec_fft;
      * benches/ec_fft.rs:62-112: 32 concurrent tasks of a forward + inverse
        2^6 transform on their own contexts; check: output = n x input.
    Timings are best of 3 after one warm call (the reference prints one)."""
    import threading

    cid = ecgpu.CURVE_NAMES[curve]
    lq = ecgpu.CURVE_FQ_LIMBS[cid]
    r_int = R_BLS if cid == 0 else R_BN
    out = {"curve": curve}

    def best_of(fn, k=3):
        fn()
        b = 1e9
        for _ in range(k):
            t = time.perf_counter()
            fn()
            b = min(b, time.perf_counter() - t)
        return b

    # ---- benches/multiexp.rs
    n = 1 << 22
    hb = np.ascontiguousarray(np.resize(co.gen_bases(cid, 41, 43, 99), (n, 2 * lq)))
    he = np.ascontiguousarray(np.resize(rand_scalars(np.random.default_rng(73), 73, r_int), (n, 4)))
    d_b = ecgpu.upload_multiexp_bases(prog, hb, curve=curve)
    d_e = ecgpu.DeviceBuffer.upload(prog, he)
    res = {}

    def mm():
        res["o"] = ecgpu.multiple_multiexp(prog, d_b, (d_e, n), 1024, 8, False, curve=curve)

    s = best_of(mm)
    want = co.multiexp_cpu(cid, hb, he, nthreads=nthreads)
    out["multiexp"] = {"shape": "2^22 terms (bases period 99, scalars period 73), 1024 tasks of 4096, window 8",
                       "ms": s * 1e3, "terms_per_s": n / s,
                       "equal": _same_point(co, cid, _fold_points(co, cid, res["o"]), want)}
    d_b.free()
    d_e.free()
    del hb, he
    # ---- benches/amt.rs
    L, lines = 1 << 21, 10
    hb = np.ascontiguousarray(np.resize(co.gen_bases(cid, 7, 11, 97), (L * lines, 2 * lq)))
    he = np.ascontiguousarray(np.resize(rand_scalars(np.random.default_rng(173), 73, r_int), (L, 4)))
    d_b = ecgpu.upload_multiexp_bases(prog, hb, curve=curve)
    d_e = ecgpu.DeviceBuffer.upload(prog, he)
    sweep, line_sums = {}, None
    equal = True
    for gd in range(7, 12):
        groups = 1 << gd

        def amt():
            res["o"] = ecgpu.multiple_multiexp(prog, d_b, (d_e, L), groups, 8, True, curve=curve)

        sweep[str(gd)] = best_of(amt) * 1e3
        sums = [_fold_points(co, cid, res["o"][ln * groups:(ln + 1) * groups]) for ln in range(lines)]
        if line_sums is None:
            line_sums = sums
            equal = equal and _same_point(co, cid, sums[0], co.multiexp_cpu(cid, hb[:L], he, nthreads=nthreads))
        else:
            equal = equal and all(_same_point(co, cid, a, b) for a, b in zip(sums, line_sums))
    out["amt"] = {"shape": f"{lines} lines x 2^21 terms (bases period 97, scalars period 73)",
                  "ms_by_group_degree": sweep, "terms_per_s_best": L * lines / (min(sweep.values()) / 1e3),
                  "equal": bool(equal)}
    # the bench's full grid (amt.rs:38-56): every group degree x window size
    # 4..9, the window pinned as the reference kernel takes it (pin_window)
    grid, eq_grid = {}, True
    for gd in range(7, 12):
        groups = 1 << gd
        row = {}
        for ws in range(4, 10):
            def amt_w():
                res["o"] = ecgpu.multiple_multiexp(prog, d_b, (d_e, L), groups, ws, True, curve=curve,
                                                   pin_window=True)

            row[str(ws)] = best_of(amt_w, 1) * 1e3
            sums = [_fold_points(co, cid, res["o"][ln * groups:(ln + 1) * groups]) for ln in range(lines)]
            eq_grid = eq_grid and all(_same_point(co, cid, a, b) for a, b in zip(sums, line_sums))
        grid[str(gd)] = row
    out["amt_window_grid"] = {"ms_by_group_degree_and_window": grid, "equal": bool(eq_grid),
                              "note": "window pinned (pin_window=True) as multiple_multiexp_st(.., window_size, "
                                      "true) takes it; each cell's per-line sums == the auto-window sweep's"}
    d_b.free()
    d_e.free()
    del hb, he
    # ---- benches/ec_fft.rs (sequential): radix_ec_fft per degree 0..11, host points
    p_mod = P_BLS if cid == 0 else P_BN
    one = u64(((1 << (64 * lq)) % p_mod), lq)
    aff = co.gen_bases(cid, 3, 7, 1 << 11)
    jac = np.ascontiguousarray(np.concatenate([aff, np.tile(one, (1 << 11, 1))], axis=1))
    ek = ecgpu.EcFftKernel.create([prog], curve)
    seq, eq_seq = {}, True
    for deg in range(12):
        x = np.ascontiguousarray(jac[:1 << deg])
        om = omega_for(cid, r_int, deg)

        def one_fft():
            y = x.copy()
            ek.radix_ec_fft(y, om, deg)
            res["o"] = y

        seq[str(deg)] = best_of(one_fft) * 1e3
        ref = co.serial_ec_fft(cid, x, om, deg, nthreads=nthreads)
        eq_seq = eq_seq and all(_same_point(co, cid, a, b) for a, b in zip(res["o"], ref))
    out["ec_fft_sequential"] = {"ms_by_log_n": seq, "equal": bool(eq_seq)}
    # ---- benches/ec_fft.rs (parallel): 32 threads, forward + inverse 2^6 each on its own context
    ln6, tasks = 6, 32
    om6 = omega_for(cid, r_int, ln6)
    w6 = int(sum(int(v) << (64 * i) for i, v in enumerate(om6))) * pow(1 << 256, -1, r_int) % r_int
    om6_inv = u64(pow(w6, -1, r_int) * (1 << 256) % r_int)
    tprogs = [ecgpu.program(ecgpu.Device(dev_index)) for _ in range(tasks)]
    tks = [ecgpu.EcFftKernel.create([tp], curve) for tp in tprogs]
    xs = [np.ascontiguousarray(jac[(i % 32) << ln6:((i % 32) + 1) << ln6]) for i in range(tasks)]

    def par_round():
        ys = [x.copy() for x in xs]

        def task(i):
            tks[i].radix_ec_fft(ys[i], om6, ln6)
            tks[i].radix_ec_fft(ys[i], om6_inv, ln6)

        th = [threading.Thread(target=task, args=(i,)) for i in range(tasks)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        res["o"] = ys

    ps = best_of(par_round)
    n6 = co.u64arr([1 << ln6], 4)
    ok = all(_same_point(co, cid, res["o"][i][j], co.naive_multiexp(cid, np.ascontiguousarray(xs[i][j:j + 1, :2 * lq]), n6))
             for i in (0, tasks - 1) for j in range(1 << ln6))
    for tp in tprogs:
        tp.close()
    out["ec_fft_parallel"] = {"tasks": tasks, "log_n": ln6, "ms": ps * 1e3, "forward_inverse_is_n_times_input": bool(ok)}
    return out


def _g2_kat(cid: int, scal: np.ndarray, r_int: int, got: np.ndarray) -> bool:
    """sum_j s_j (KAT_A + j KAT_B) G2 through the Python G2 restatement (checker only)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as co
    import py_oracle as po

    cv = po.BLS12_381_G2 if cid == 0 else po.BN254_G2
    k = co.kat_scalar(cid, KAT_A % r_int, KAT_B, scal, nthreads=cpu_threads(0))
    want = po.g2_to_affine(cv, po.g2_scalar_mul(cv, cv.gen, k))
    n, p = cv.fq.limbs64, cv.fq.modulus
    j = np.asarray(got).reshape(3, 2 * n)

    def fq2(limbs):
        return po.Fq2(cv.fq.from_mont(po.limbs_to_int(limbs[:n])), cv.fq.from_mont(po.limbs_to_int(limbs[n:])), p)

    return po.jac_to_affine((fq2(j[0]), fq2(j[1]), fq2(j[2])), p) == want


def pmc_traffic(kernel: str):
    """HBM bytes per launch (GB) from the committed rocprofv3 PMC passes
    (tools/gpu.sh prof -> profiles/<round>/pmc_fetch_write.json, copied to
    profiles/pmc_current.json with its source): 2 x FETCH_SIZE + WRITE_SIZE.
    gfx950 FETCH_SIZE tallies each 128-B read request at 64 B (TCC_EA0_RDREQ
    x 64; MI355X_MICROARCH.md, HBM/rocprofv3 section), so it is doubled for
    both kernels: the NTT's 16-B/lane streaming reads and the accumulation's
    16-B/lane reads of whole 128-B base records are both 128-B requests."""
    path = os.path.join(ROOT, "profiles", "pmc_current.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            d = json.load(f)
        for k, v in d["kernels"].items():
            if kernel in k:
                fetch = v["FETCH_SIZE"]["mean_kb"] * 1024 / 1e9
                write = v["WRITE_SIZE"]["mean_kb"] * 1024 / 1e9
                return 2 * fetch + write, d["source"]
    except (OSError, ValueError, KeyError, TypeError) as e:  # a malformed record must not sink the bench line
        print(f"bench: ignoring {path}: {type(e).__name__}: {e}", file=sys.stderr)
    return None, None


if __name__ == "__main__":
    main()
