"""world_size-2 multi-process test (gloo on CPU) of the sharded MSM
orchestration used by bench.py on N GPUs: contiguous range shards, all-gather
of the per-rank partial points, fold.  On the GPU the partials come from
ecg_msm_dev and the fold from ecg_point_sum_dev over RCCL; here both are the
CPU oracle so the orchestration itself is what is tested."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
    import torch
    import torch.distributed as dist

    import coracle as co
    import py_oracle as po
    from ecgpu.dist import msm_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cid, n = 0, 777
        rng = po.Xoshiro256ss(4242)  # same inputs on every rank
        B = co.gen_bases(cid, 31, 37, n, 2)
        E = co.u64arr([rng.field_element(po.BLS12_381_FR) for _ in range(n)], 4)

        def partial(i0, i1):
            p = co.multiexp_cpu(cid, B[i0:i1], E[i0:i1], nthreads=2) if i1 > i0 else \
                co.u64arr([0, 1, 0], 6).reshape(-1)  # identity (0, 1, 0)
            if i1 > i0:
                p = p.reshape(-1)
            return torch.from_numpy(p.view(np.int64).copy())

        def fold(parts):
            acc = np.zeros(18, dtype=np.uint64)
            acc[6:12] = co.u64arr([1], 6)[0]  # placeholder y; z = 0 means identity
            for t in parts:
                p = t.numpy().view(np.uint64).copy()
                co.lib().orc_jac_add(cid, co.ptr(acc), co.ptr(acc), co.ptr(p))
            return acc

        got = msm_sharded(n, partial, fold)
        want = co.multiexp_cpu(cid, B, E, nthreads=2)
        ok = bool((co.jac_to_affine(cid, got) == co.jac_to_affine(cid, want)).all())
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_msm_sharded_gloo_world2():
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    results = dict(q.get(timeout=10) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    assert results == {0: True, 1: True}
