"""Multi-GPU sharding for the MSM + FFT path: one process per GPU.

Reference behaviour being replaced (ec-gpu-proxy):
  * MultiexpKernel::parallel_multiexp (src/multiexp.rs:324-367) splits the
    terms into ceil(N / #devices) contiguous ranges, one host thread per
    device, then sums the per-device results on the host (multiexp.rs:394-397).
  * FftKernel::radix_fft_many (src/fft.rs:211-246) gives each device a
    contiguous chunk of ceil(m / #devices) whole transforms (no exchange).

Here every rank owns one GPU.  MSM: each rank computes the partial sum of its
range on its own GPU, the partials (one normalised Jacobian point, 144 B for
BLS12-381) are all-gathered with RCCL over xGMI -- RCCL has no elliptic-curve
reduction op -- and folded (ecg_msm_dist).  FFT: whole transforms are
assigned by chunk; nothing is exchanged.  One transform too large for a GPU,
or already block-distributed, runs as ecg_fft_dist (three RCCL all-to-alls,
dfft.hip).

RCCL lives inside libecgpu, on the ROCm install's HIP runtime (the same one
as its device buffers).  The host side of a launch -- the 128-byte RCCL id,
barriers, the max over ranks of a timing -- needs only a few small messages:
HostGroup carries them over one local TCP socket per rank, so a launched
process never loads a second HIP runtime (torch bundles its own copies of
libamdhip64 / librccl; importing it next to libecgpu maps both).  Any group
with a broadcast works for comm_init (torch.distributed in the gloo tests).
msm_sharded keeps the orchestration injectable so the CPU multi-process tests
exercise the same split.
"""
from __future__ import annotations

import os
import time
from typing import Any, Callable, Sequence


class HostGroup:
    """Rank 0 listens on (addr, port); every other rank connects.  Collectives
    are star-shaped through rank 0 (small host objects only: ids, timings,
    digests).  From a torch.distributed.run launch: HostGroup.from_env()."""

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29600,
                 authkey: bytes = b"ecgpu-hostgroup", timeout: float = 300.0):
        from multiprocessing.connection import Client, Listener

        if world <= 0 or not (0 <= rank < world):
            raise ValueError("bad world/rank")
        self.rank, self.world = rank, world
        self._peers = []
        self._conn = None
        self._listener = None
        if world == 1:
            return
        if rank == 0:
            self._listener = Listener((addr, port), authkey=authkey)
            peers = {}
            while len(peers) < world - 1:
                c = self._listener.accept()
                r = c.recv()
                peers[r] = c
            self._peers = [peers[r] for r in range(1, world)]
        else:
            deadline = time.time() + timeout
            while True:
                try:
                    self._conn = Client((addr, port), authkey=authkey)
                    break
                except (ConnectionRefusedError, FileNotFoundError, OSError):
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            self._conn.send(rank)

    @staticmethod
    def from_env(offset: int = 1) -> "HostGroup":
        """RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as torch.distributed.run
        sets them; the group listens on MASTER_PORT + offset (the launcher's
        own store holds MASTER_PORT)."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + offset
        return HostGroup(rank, world, addr, port)

    def allgather(self, obj: Any) -> list:
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [c.recv() for c in self._peers]
            for c in self._peers:
                c.send(out)
            return out
        self._conn.send(obj)
        return self._conn.recv()

    def broadcast(self, obj: Any = None) -> Any:
        """rank 0's obj on every rank."""
        if self.world == 1:
            return obj
        if self.rank == 0:
            for c in self._peers:
                c.send(obj)
            return obj
        return self._conn.recv()

    def barrier(self) -> None:
        self.allgather(None)

    def max(self, x: float) -> float:
        return max(self.allgather(float(x)))

    def close(self) -> None:
        for c in self._peers:
            c.close()
        if self._conn is not None:
            self._conn.close()
        if self._listener is not None:
            self._listener.close()
        self._peers, self._conn, self._listener = [], None, None


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous range of rank `rank` (multiexp.rs:332-336: chunk = ceil(n / world))."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    chunk = (n + world - 1) // world if n else 0
    i0 = min(n, rank * chunk)
    return i0, min(n, i0 + chunk)


def fft_assignment(count: int, world: int) -> list[list[int]]:
    """Transform indices per device (fft.rs:216-225: chunks of ceil(m / #dev))."""
    if count == 0:
        return [[] for _ in range(world)]
    chunk = (count + world - 1) // world
    return [list(range(min(count, d * chunk), min(count, (d + 1) * chunk))) for d in range(world)]


def msm_sharded(n: int, partial_fn: Callable[[int, int], "object"], fold_fn: Callable[[Sequence], "object"],
                group=None):
    """Sharded MSM over the default (or given) torch.distributed group.

    partial_fn(i0, i1) -> this rank's partial point as a 1-D int64 tensor on
    the collective's device (3*Lq limbs).  fold_fn(list_of_partials) -> the
    folded result.  Every rank returns the same folded value."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    i0, i1 = shard_range(n, world, rank)
    part = partial_fn(i0, i1)
    if not isinstance(part, torch.Tensor):
        raise TypeError("partial_fn must return a torch.Tensor")
    gathered = [torch.zeros_like(part) for _ in range(world)]
    dist.all_gather(gathered, part, group=group)
    return fold_fn(gathered)


# ---------------------------------------------------------------------------
# native RCCL path (libecgpu ecg_comm_* / ecg_msm_dist / ecg_fft_dist)
# ---------------------------------------------------------------------------


def comm_init(prog, rank: int, world: int, broadcast: Callable[[Any], Any] | None = None,
              make_id: Callable[[], bytes] | None = None) -> None:
    """Rank 0 makes the RCCL id (make_id, default ecg_comm_unique_id), the
    launcher's group broadcasts it (broadcast(obj) -> rank 0's obj, e.g.
    HostGroup.broadcast), every rank binds its Program's context
    (ecg_comm_init).  make_id is injectable so the CPU tests run the same
    exchange without RCCL."""
    import ctypes

    import ecgpu

    buf = (ctypes.c_uint8 * 128)()
    if world > 1:
        ident = None
        if rank == 0:
            ident = make_id() if make_id is not None else unique_id()
        ident = broadcast(ident)
        if not isinstance(ident, (bytes, bytearray)) or len(ident) != 128:
            raise ValueError("comm_init: the broadcast RCCL id must be 128 bytes")
        ctypes.memmove(buf, bytes(ident), 128)
    if prog is None:  # exchange only (CPU tests)
        return bytes(buf)
    ecgpu._check(ecgpu.lib().ecg_comm_init(prog.handle, world, rank, buf), "comm_init")
    return bytes(buf)


def unique_id() -> bytes:
    import ctypes

    import ecgpu

    buf = (ctypes.c_uint8 * 128)()
    ecgpu._check(ecgpu.lib().ecg_comm_unique_id(buf), "comm_unique_id")
    return bytes(buf)


def torch_broadcast(dist_mod=None, group=None) -> Callable[[Any], Any]:
    """broadcast(obj) over a torch.distributed group (gloo tests)."""
    if dist_mod is None:
        import torch.distributed as dist_mod

    def bcast(obj):
        lst = [obj]
        dist_mod.broadcast_object_list(lst, src=0, group=group)
        return lst[0]

    return bcast


def msm_dist(prog, curve, d_bases, d_scalars, n_local: int):
    """This rank's shard + RCCL all-gather of partials + fold -> full result."""
    import numpy as np

    import ecgpu

    cid = ecgpu._curve(curve)
    out = np.zeros(3 * ecgpu.CURVE_FQ_LIMBS[cid], dtype=np.uint64)
    ecgpu._check(ecgpu.lib().ecg_msm_dist(prog.handle, cid, d_bases.ptr, d_scalars.ptr, n_local, ecgpu._ptr(out)),
                 "msm_dist")
    return out


def fft_dist(prog, field, d_local, omega, log_n: int) -> None:
    """One 2^log_n NTT, block-distributed over the communicator (in place)."""
    import numpy as np

    import ecgpu

    om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
    ecgpu._check(ecgpu.lib().ecg_fft_dist(prog.handle, ecgpu._fft_field(field), d_local.ptr, ecgpu._ptr(om), log_n),
                 "fft_dist")


def fft_dist_emulated(progs, field, d_blocks, omega, log_n: int) -> None:
    """ecg_fft_dist's schedule for T block-buffers held in one process (one
    context each, e.g. all on one GPU): the three all-to-alls are done by
    host copies, the local steps by the same device kernels
    (ecg_fft_dist_stage1/3, ecg_fft_dev).  Test and rehearsal harness for the
    multi-rank path on a single-GPU box."""
    import numpy as np

    import ecgpu

    T = len(d_blocks)
    fid = ecgpu._fft_field(field)
    lib = ecgpu.lib()
    m = (1 << log_n) // T
    seg = m // T
    om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)

    def all_to_all(bufs):
        host = [b.read(shape=(T, seg, 4)) for b in bufs]
        for q in range(T):
            bufs[q].write(np.ascontiguousarray(np.stack([host[s][q] for s in range(T)])))

    tmp = [ecgpu.DeviceBuffer(p, m * 32) for p in progs]
    all_to_all(d_blocks)
    for r in range(T):
        ecgpu._check(lib.ecg_fft_dist_stage1(progs[r].handle, fid, d_blocks[r].ptr, tmp[r].ptr, ecgpu._ptr(om),
                                             T, r, log_n), "fft_dist_stage1")
    all_to_all(tmp)
    # local m-point NTT with omega^T
    r_mod = {0: 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
             2: 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001}[fid]
    w = sum(int(om[i]) << (64 * i) for i in range(4)) * pow(1 << 256, -1, r_mod) % r_mod
    wt = pow(w, T, r_mod) * (1 << 256) % r_mod
    om_t = np.array([(wt >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
    for r in range(T):
        ecgpu.fft_dev(progs[r], field, tmp[r], om_t, log_n - (T.bit_length() - 1))
    all_to_all(tmp)
    for r in range(T):
        ecgpu._check(lib.ecg_fft_dist_stage3(progs[r].handle, tmp[r].ptr, d_blocks[r].ptr, T, log_n),
                     "fft_dist_stage3")
    for t in tmp:
        t.free()
