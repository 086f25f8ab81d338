"""world_size-2 multi-process CPU tests of the N>1 path bench.py runs.

* test_bench_main_world2: two processes run bench.main() itself under the
  launcher's environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
  MASTER_PORT, as torch.distributed.run sets them): HostGroup.from_env on
  MASTER_PORT + 1, comm_init's id broadcast, the per-rank shards and seeds,
  the barrier / max-over-ranks timing, rank 0's full-size KAT regeneration,
  the distributed-NTT digest check and the rank-0-only JSON report.  Only the
  device calls (program, DeviceBuffer, gen_bases_dev, prepare_bases, msm_dev,
  fft_dev, msm_dist, fft_dist) are replaced, by CPU-oracle stand-ins that
  exchange partials and blocks over a second HostGroup as RCCL would.
* test_bench_dist_path_world2: two processes run bench.py's own host-side
  orchestration -- ecgpu.dist.HostGroup (the launch's control channel),
  comm_init's RCCL-id broadcast (with an injected id maker: no RCCL on CPU),
  bench.msm_shard's contiguous shards and seeds, the all-gather of per-rank
  partial points and their fold, the max-over-ranks timing reduction, and
  bench.msm_kat_scalar's full-size known answer regenerated on rank 0.  The
  per-rank partial comes from the CPU oracle instead of ecg_msm_dist.
* test_msm_sharded_gloo_world2: the same split through torch.distributed over
  gloo (ecgpu.dist.msm_sharded / torch_broadcast)."""
import json
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _fold(co, cid, parts):
    nq = 6 if cid == 0 else 4
    acc = np.zeros(3 * nq, dtype=np.uint64)
    for p in parts:
        p = np.ascontiguousarray(p, dtype=np.uint64)
        co.lib().orc_jac_add(cid, co.ptr(acc), co.ptr(acc), co.ptr(p))
    return acc


def _bench_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
    import bench
    import coracle as co
    from ecgpu import dist as edist

    group = edist.HostGroup(rank, world, "127.0.0.1", port)
    try:
        ident = edist.comm_init(None, rank, world, group.broadcast, make_id=lambda: bytes(range(128)))
        ids = group.allgather(ident)
        ok_id = all(i == bytes(range(128)) for i in ids)
        for cid, r_int in ((0, bench.R_BLS), (1, bench.R_BN)):
            n_total = 1001
            i0, n_loc, scal, a_loc = bench.msm_shard(rank, world, n_total, r_int)
            assert (i0, i0 + n_loc) == edist.shard_range(n_total, world, rank)
            B = co.gen_bases(cid, a_loc, bench.KAT_B, n_loc, 2)
            part = co.multiexp_cpu(cid, B, scal, nthreads=2).reshape(-1)
            parts = group.allgather(part)
            got = _fold(co, cid, parts)
            if rank == 0:
                kat = bench.msm_kat_scalar(co, cid, world, n_total, r_int, 2)
                want = co.gen_mul(cid, kat)
                ok_id = ok_id and bool((co.jac_to_affine(cid, got) == co.jac_to_affine(cid, want)).all())
        t = group.max(0.5 + rank)
        group.barrier()
        q.put((rank, ok_id and t == 0.5 + world - 1))
    finally:
        group.close()


@pytest.mark.timeout(300)
def test_bench_dist_path_world2():
    import multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    results = dict(q.get(timeout=10) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    assert results == {0: True, 1: True}


class _FakeProg:
    handle = None

    def synchronize(self):
        pass

    def kernel_time(self, name):
        return 0.25, 1


class _FakeBuf:
    """DeviceBuffer stand-in: the 'device' bytes are a numpy array."""

    def __init__(self, arr):
        self.arr = np.ascontiguousarray(arr, dtype=np.uint64).copy()
        self.ptr = id(self)
        self.nbytes = self.arr.nbytes

    @staticmethod
    def upload(prog, host):
        return _FakeBuf(host)

    def write(self, host):
        self.arr[...] = np.asarray(host, dtype=np.uint64).reshape(self.arr.shape)

    def read(self, dtype=np.uint64, shape=None):
        out = self.arr.copy()
        return out.reshape(shape) if shape is not None else out

    def free(self):
        self.ptr = None


def _install_device_fakes(rank, world, corrupt=False, fail_rank=None):
    """Swap ecgpu's device entry points for CPU-oracle stand-ins (checker-grade
    results, so bench.main()'s own checks can pass or fail for real).
    msm_dist follows ecg_msm_dist_ex's protocol (comm.cpp): every rank
    all-gathers a [status, partial] record, and any failed status -- here
    rank `fail_rank` emulating a local allocation failure -- raises the lowest
    failing rank's error on EVERY rank instead of leaving peers waiting."""
    import coracle as co
    import ecgpu
    from ecgpu import dist as edist

    side = edist.HostGroup.from_env(offset=2)  # the 'RCCL' of the stand-ins
    real_comm_init = edist.comm_init
    fid_of = {"bls12_381_fr": 0, "bn254_fr": 2}

    def gen_bases_dev(prog, curve, a, b, n):
        return _FakeBuf(co.gen_bases(ecgpu._curve(curve), int(a), int(b), n, 2))

    def msm_local(curve, bases, scal, n):
        cid = ecgpu._curve(curve)
        nq = ecgpu.CURVE_FQ_LIMBS[cid]
        if n == 0:
            return np.concatenate([np.zeros(nq, np.uint64), co.u64arr([1], nq)[0], np.zeros(nq, np.uint64)])
        return co.multiexp_cpu(cid, bases.arr.reshape(-1, 2 * nq)[:n], scal.arr.reshape(-1, 4)[:n],
                               nthreads=2).reshape(-1)

    def msm_dist(prog, curve, bases, scal, n_local, maybe_abort=None):
        cid = ecgpu._curve(curve)
        if rank == fail_rank:
            rec = [ecgpu.ECG_ERR_NOMEM, None]
        elif maybe_abort is not None and maybe_abort():
            rec = [ecgpu.ECG_ABORTED, None]
        else:
            rec = [ecgpu.ECG_OK, msm_local(curve, bases, scal, n_local)]
        recs = side.allgather(rec)
        for r, (rc, _) in enumerate(recs):
            if rc != ecgpu.ECG_OK:
                if rc == ecgpu.ECG_ABORTED:
                    raise ecgpu.Aborted("GPU call was aborted!")
                raise ecgpu.EcError(f"msm_dist: ecg_msm_dist: rank {r} of {world} failed (rc={rc}); every rank stops")
        return _fold(co, cid, [p for _, p in recs])

    def msm_dist_grid(prog, curve, bases, scal, n, maybe_abort=None):
        # every rank holds all n terms; this stand-in's "1/N of the grid" is a
        # term range of them (the partials fold to the same total)
        cid = ecgpu._curve(curve)
        nq = ecgpu.CURVE_FQ_LIMBS[cid]
        assert bases.arr.size == n * 2 * nq and scal.arr.size == n * 4, "grid split needs replicated operands"
        i0, i1 = edist.shard_range(n, world, rank)
        sub_b, sub_s = _FakeBuf(bases.arr.reshape(-1, 2 * nq)[i0:i1]), _FakeBuf(scal.arr.reshape(-1, 4)[i0:i1])
        return msm_dist(prog, curve, sub_b, sub_s, i1 - i0, maybe_abort)

    def fft_dev(prog, field, d, omega, log_n):
        d.arr[...] = co.serial_fft(fid_of[field], d.arr.reshape(-1, 4), np.asarray(omega, np.uint64), log_n)

    def fft_dist(prog, field, d_local, omega, log_n):
        blocks = side.allgather(d_local.arr.reshape(-1, 4))
        full = co.serial_fft(fid_of[field], np.ascontiguousarray(np.concatenate(blocks)),
                             np.asarray(omega, np.uint64), log_n)
        m = full.shape[0] // world
        d_local.arr[...] = full[rank * m:(rank + 1) * m]
        if corrupt and rank == 1:
            d_local.arr.reshape(-1)[5] ^= np.uint64(1)

    ecgpu.Device = lambda i: i
    ecgpu.program = lambda dev: _FakeProg()
    ecgpu.DeviceBuffer = _FakeBuf
    ecgpu.gen_bases_dev = gen_bases_dev
    ecgpu.prepare_bases = lambda prog, curve, d, n, window_table=None: d
    ecgpu.msm_dev = lambda prog, curve, b, s, n: msm_local(curve, b, s, n)
    ecgpu.fft_dev = fft_dev
    edist.comm_init = lambda prog, r, w, bcast, **kw: real_comm_init(None, r, w, bcast,
                                                                     make_id=lambda: bytes(range(128)))
    edist.msm_dist = msm_dist
    edist.msm_dist_grid = msm_dist_grid
    edist.fft_dist = fft_dist
    # what an RCCL communicator of `world` ranks on distinct devices reports
    edist.comm_info = lambda prog: {"count": world, "rank": rank, "device": rank,
                                    "pci_bus_id": f"0000:{0x11 + 0x10 * rank:02x}:00.0", "transport": "rccl"}
    edist.last_exchange_us = lambda prog: 40.0 + rank
    return side


def _bench_main_worker(rank, world, port, q, corrupt=False, fail_rank=None, extra=()):
    import contextlib
    import io

    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "OMP_NUM_THREADS": "2"})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
    side = _install_device_fakes(rank, world, corrupt, fail_rank)
    import bench
    import ecgpu

    sys.argv = ["bench.py", "--gpus", str(world), "--steps", "2", "--warmup", "1", "--msm-log", "10",
                "--ntt-log", "8", *extra]
    out = io.StringIO()
    try:
        with contextlib.redirect_stdout(out):
            bench.main()
    except ecgpu.EcError as e:  # the failure reached this rank: report it and exit non-zero
        q.put((rank, "ERROR " + str(e) + "\n" + out.getvalue()))
        side.close()
        sys.exit(3)
    finally:
        side.close()
    q.put((rank, out.getvalue()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("corrupt", [False, True], ids=["exact", "corrupted_block"])
def test_bench_main_world2(corrupt):
    """bench.main() end to end at N = 2 on CPU: the JSON line rank 0 prints
    carries the full-size MSM KAT and the distributed-NTT digest check; one
    flipped bit in rank 1's NTT block turns exactly that check false."""
    import json
    import multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_main_worker, args=(r, 2, port, q, corrupt)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    outs = dict(q.get(timeout=10) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    assert outs[1] == ""  # only rank 0 reports
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["msm_terms"] == 1 << 10
    assert line["checks"] == {"msm_kat_2^10": True, "ntt_vs_parallel_fft_2^8": True,
                              "ntt_dist_2gpu_vs_parallel_fft_2^8": not corrupt}
    assert line["value"] > 0 and line["ntt_dist"]["value"] > 0
    assert line["msm_window_table"]["equals_headline_result"] is True
    # rank 0's record of what every rank's communicator reported
    assert line["rccl"] == {"transport": ["rccl"], "count": [2], "ranks": [0, 1],
                            "devices": ["0000:11:00.0", "0000:21:00.0"], "distinct": True,
                            "msm_allgather_us": 41.0}


@pytest.mark.timeout(300)
def test_bench_main_world2_grid_split():
    """bench.main() at N = 2 with --msm-split grid: every rank generates all
    2^10 bases and the scalars of both shards, the JSON line records the split
    and the full-size KAT holds."""
    import multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_main_worker, args=(r, 2, port, q, False, None, ("--msm-split", "grid")))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    outs = dict(q.get(timeout=10) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["config"]["msm_split"] == "grid" and "grid split" in line["config"]["parallelism"]
    assert line["checks"]["msm_kat_2^10"] is True
    assert line["msm_window_table"] is None


@pytest.mark.timeout(300)
def test_bench_main_world4_auto_split():
    """bench.main() at N = 4 with the default --msm-split auto: BLS12-381 takes
    the grid split from N = 4 on; the KAT and the NTT digests
    hold and the line records the split."""
    import multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_main_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(280)
    outs = dict(q.get(timeout=10) for _ in range(4))
    assert all(p.exitcode == 0 for p in procs)
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["n_gpus"] == 4 and line["config"]["msm_split"] == "grid"
    assert line["checks"]["msm_kat_2^10"] is True and line["checks"]["ntt_dist_4gpu_vs_parallel_fft_2^8"] is True


@pytest.mark.timeout(300)
def test_bench_main_world2_failing_rank():
    """bench.main() at N = 2 with rank 1's distributed MSM failing locally
    (an emulated allocation failure inside ecg_msm_dist): the status rides in
    the all-gather, so BOTH ranks raise at that call -- nobody is left in the
    exchange, both processes exit non-zero well within the timeout, and rank 0
    prints no JSON line."""
    import multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_main_worker, args=(r, 2, port, q, False, 1)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert not any(p.is_alive() for p in procs), "a rank hung after its peer failed"
    outs = dict(q.get(timeout=10) for _ in range(2))
    assert [p.exitcode for p in procs] == [3, 3]
    assert outs[0].startswith("ERROR") and "rank 1 of 2 failed" in outs[0]
    assert outs[1].startswith("ERROR") and "rank 1 of 2 failed" in outs[1]
    assert '"metric"' not in outs[0]


def _run_self_launch(world, extra_env=None, timeout=280):
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update({"OMP_NUM_THREADS": "2", **(extra_env or {})})
    cmd = [sys.executable, os.path.join(ROOT, "tests", "bench_fake_ranks.py"), "--gpus", str(world),
           "--steps", "2", "--warmup", "1", "--msm-log", "10", "--ntt-log", "8"]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(300)
def test_bench_self_launch_world2():
    """`bench.py --gpus 2` without torch.distributed.run: the process starts its
    two rank processes itself (bench.launch_ranks), and exactly one JSON line
    -- rank 0's -- comes out, recording both ranks' communicators."""
    p = _run_self_launch(2)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["rccl"]["count"] == [2]
    assert line["rccl"]["ranks"] == [0, 1] and line["rccl"]["distinct"] is True
    assert line["checks"]["msm_kat_2^10"] is True and line["checks"]["ntt_dist_2gpu_vs_parallel_fft_2^8"] is True


@pytest.mark.timeout(300)
def test_bench_self_launch_failing_rank():
    """A rank that fails makes the launching process exit non-zero, with no
    JSON line and no rank left running."""
    p = _run_self_launch(2, {"FAKE_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert '"metric"' not in p.stdout
    assert "rank 1 of 2 failed" in p.stderr


def test_kat_scalar_regeneration_matches_single_rank():
    """bench.msm_kat_scalar over 3 regenerated shards == the KAT of the
    concatenated scalars: the N>1 check covers exactly the full workload."""
    sys.path.insert(0, ROOT)
    import bench
    import coracle as co

    n, world = 1000, 3
    shards = [bench.msm_shard(r, world, n, bench.R_BLS) for r in range(world)]
    allsc = np.ascontiguousarray(np.concatenate([s[2] for s in shards]))
    assert allsc.shape == (n, 4)
    k1 = bench.msm_kat_scalar(co, 0, world, n, bench.R_BLS, 2)
    k2 = co.kat_scalar(0, bench.KAT_A, bench.KAT_B, allsc, nthreads=2)
    assert k1 == k2


def test_bench_reads_committed_pmc_records():
    """The committed PMC summaries the default bench line quotes as
    roofline.traffic parse (a reshaped file once sank a round-end bench)."""
    sys.path.insert(0, ROOT)
    import bench

    for kernel in ("msm_accumulate", "ntt_pass"):
        gb, src = bench.pmc_traffic(kernel)
        assert gb is not None and gb > 0 and src.startswith("profiles/"), kernel
    with open(os.path.join(ROOT, "profiles", "pmc_bn254_current.json")) as f:
        d = json.load(f)
    assert d["traffic_gb_per_launch"] > 0 and d["source"].startswith("profiles/")
    assert d["ntt_traffic_gb_per_launch"] > 0 and d["ntt_source"].startswith("profiles/")


def _gloo_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
    import torch
    import torch.distributed as dist

    import coracle as co
    import py_oracle as po
    from ecgpu.dist import comm_init, msm_sharded, torch_broadcast

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ident = comm_init(None, rank, world, torch_broadcast(dist), make_id=lambda: b"\x07" * 128)
        cid, n = 0, 777
        rng = po.Xoshiro256ss(4242)  # same inputs on every rank
        B = co.gen_bases(cid, 31, 37, n, 2)
        E = co.u64arr([rng.field_element(po.BLS12_381_FR) for _ in range(n)], 4)

        def partial(i0, i1):
            p = co.multiexp_cpu(cid, B[i0:i1], E[i0:i1], nthreads=2).reshape(-1) if i1 > i0 else \
                co.u64arr([0, 1, 0], 6).reshape(-1)  # identity (0, 1, 0)
            return torch.from_numpy(p.view(np.int64).copy())

        def fold(parts):
            return _fold(co, cid, [t.numpy().view(np.uint64) for t in parts])

        got = msm_sharded(n, partial, fold)
        want = co.multiexp_cpu(cid, B, E, nthreads=2)
        ok = bool((co.jac_to_affine(cid, got) == co.jac_to_affine(cid, want)).all())
        q.put((rank, ok and ident == b"\x07" * 128))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_msm_sharded_gloo_world2():
    import torch.multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    results = dict(q.get(timeout=10) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    assert results == {0: True, 1: True}
