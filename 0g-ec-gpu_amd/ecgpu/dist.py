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

import hashlib
import json
import os
import time
from typing import Any, Callable, Sequence


class HostGroup:
    """Rank 0 listens on (addr, port); every other rank connects.  Collectives
    are star-shaped through rank 0 (small host values only: the RCCL id,
    timings, digests).  From a torch.distributed.run launch: HostGroup.from_env().

    Wire format: length-prefixed JSON frames (None / bool / int / float / str /
    bytes / lists / str-keyed dicts) -- nothing received is ever unpickled or
    executed.

    Authentication is mutual and covers every frame.  Rank 0 sends a random
    challenge c0; the joining peer answers with its rank, its own challenge c1
    and HMAC-SHA256(key, "join" | c0 | c1 | rank); rank 0 answers with
    HMAC(key, "accept" | c0 | c1 | rank), so the peer also knows it reached a
    holder of the key (not a process that took the port first).  Both derive a
    session key HMAC(key, "session" | c0 | c1 | rank), and every later frame
    carries HMAC(session, direction | sequence number | payload): a frame that
    was forged, altered, replayed or reordered is refused (ConnectionError).

    The key is ECGPU_HOSTGROUP_KEY when set.  Without it, a single-node launch
    (LOCAL_WORLD_SIZE == WORLD_SIZE, rank 0 bound to loopback) uses a random
    key: rank 0 writes it, before it listens, into a file of this user's 0700
    directory ($XDG_RUNTIME_DIR or the temp dir, `ecgpu-<uid>`), each peer reads
    it once rank 0 has answered its connection, and rank 0 removes it when every
    rank has joined -- so another local user can neither read the key nor plant
    one, where a key derived from the launch's public run id and port could be
    computed by anyone on the host; a multi-node launch, whose
    rank 0 listens on MASTER_ADDR, refuses to start without an explicit key
    (fail closed).  Rank 0 drops connections that fail the handshake, name an
    out-of-range or duplicate rank, or stall, and keeps accepting until every
    rank has joined or `timeout` expires."""

    _MAX_FRAME = 1 << 20

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29600,
                 key: bytes | None = None, timeout: float = 300.0, bind_addr: str | None = None):
        import socket

        if world <= 0 or not (0 <= rank < world):
            raise ValueError("bad world/rank")
        self.rank, self.world = rank, world
        self._peers: list = []
        self._conn = None
        self._listener = None
        self._timeout = timeout
        self._sess: dict = {}   # peer rank (rank 0) or 0 (peers) -> [session key, send seq, recv seq]
        if world == 1:
            return
        # the launch key: given, ECGPU_HOSTGROUP_KEY, or (single node) a random key
        # that rank 0 writes into this user's private directory before it listens
        # and the peers read once rank 0 has answered them (_key_file)
        self._key_path = None
        self._key = key if key is not None else _launch_key(port)
        if self._key is None:
            self._key_path = _key_file(port)
            if rank == 0:
                self._key = os.urandom(32)
                _write_private(self._key_path, self._key)
        deadline = time.time() + timeout
        if rank == 0:
            ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            ls.bind((bind_addr or addr, port))
            ls.listen(world)
            self._listener = ls
            peers: dict = {}
            while len(peers) < world - 1:
                left = deadline - time.time()
                if left <= 0:
                    self.close()
                    raise TimeoutError(f"HostGroup: {len(peers) + 1} of {world} ranks joined within {timeout} s")
                ls.settimeout(left)
                try:
                    c, _ = ls.accept()
                except socket.timeout:
                    continue
                r = self._admit(c, peers)
                if r is None:
                    c.close()
                    continue
                peers[r] = c
            self._peers = [peers[r] for r in range(1, world)]
            self._drop_key_file()
        else:
            while True:
                try:
                    c = socket.create_connection((addr, port), timeout=min(10.0, timeout))
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            c.settimeout(timeout)
            import hmac

            c0 = _recv_exact(c, 32)
            if self._key is None:  # rank 0 wrote it before listening
                self._key = _read_private(self._key_path)
            c1 = os.urandom(32)
            c.sendall(rank.to_bytes(4, "little") + c1 + _mac(self._key, b"join", c0, c1, rank))
            reply = _recv_exact(c, 34)
            if reply[:2] != b"ok" or not hmac.compare_digest(reply[2:], _mac(self._key, b"accept", c0, c1, rank)):
                c.close()
                raise ConnectionError("HostGroup: rank 0 refused this rank, or could not prove it holds the key")
            self._sess[0] = [_mac(self._key, b"session", c0, c1, rank), 0, 0]
            self._conn = c

    def _admit(self, c, peers: dict):
        """Mutual handshake with one connection; its rank if admitted, else None."""
        import hmac
        import socket

        try:
            c.settimeout(10.0)
            c0 = os.urandom(32)
            c.sendall(c0)
            msg = _recv_exact(c, 68)
            r = int.from_bytes(msg[:4], "little")
            c1 = msg[4:36]
            if not (1 <= r < self.world) or r in peers or not hmac.compare_digest(
                    msg[36:], _mac(self._key, b"join", c0, c1, r)):
                return None
            c.sendall(b"ok" + _mac(self._key, b"accept", c0, c1, r))
            c.settimeout(self._timeout)
            self._sess[r] = [_mac(self._key, b"session", c0, c1, r), 0, 0]
            return r
        except (OSError, socket.timeout, ConnectionError):
            return None

    @staticmethod
    def from_env(offset: int = 1) -> "HostGroup":
        """RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as torch.distributed.run
        sets them; the group listens on MASTER_PORT + offset (the launcher's
        own store holds MASTER_PORT).  On a single-node launch (LOCAL_WORLD_SIZE
        == WORLD_SIZE) rank 0 binds the loopback interface only; a multi-node
        launch needs ECGPU_HOSTGROUP_KEY (a secret every rank's environment
        shares) and refuses to start without it."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + offset
        single_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
        if world > 1 and not single_node and not os.environ.get("ECGPU_HOSTGROUP_KEY"):
            raise PermissionError("HostGroup: a multi-node launch listens on MASTER_ADDR, so it needs a secret: "
                                  "set ECGPU_HOSTGROUP_KEY to the same random value on every rank")
        bind = "127.0.0.1" if single_node else addr
        if single_node:
            addr = "127.0.0.1"
        return HostGroup(rank, world, addr, port, bind_addr=bind)

    # -- framing: length | payload | HMAC(session, direction | seq | payload)
    def _send(self, c, peer: int, obj) -> None:
        import hmac

        sess = self._sess[peer]
        data = json.dumps(_enc(obj), separators=(",", ":")).encode()
        tag = hmac.new(sess[0], b"s" + bytes([self.rank == 0]) + sess[1].to_bytes(8, "little") + data,
                       hashlib.sha256).digest()
        sess[1] += 1
        c.sendall(len(data).to_bytes(8, "little") + data + tag)

    def _recv(self, c, peer: int):
        import hmac

        sess = self._sess[peer]
        n = int.from_bytes(_recv_exact(c, 8), "little")
        if n > self._MAX_FRAME:
            raise ConnectionError(f"HostGroup: frame of {n} bytes exceeds {self._MAX_FRAME}")
        data = _recv_exact(c, n)
        tag = _recv_exact(c, 32)
        want = hmac.new(sess[0], b"s" + bytes([self.rank != 0]) + sess[2].to_bytes(8, "little") + data,
                        hashlib.sha256).digest()
        if not hmac.compare_digest(tag, want):
            raise ConnectionError("HostGroup: a frame failed authentication (forged, altered or replayed)")
        sess[2] += 1
        return _dec(json.loads(data))

    def allgather(self, obj: Any) -> list:
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [self._recv(c, r) for r, c in enumerate(self._peers, 1)]
            for r, c in enumerate(self._peers, 1):
                self._send(c, r, out)
            return out
        self._send(self._conn, 0, obj)
        return self._recv(self._conn, 0)

    def broadcast(self, obj: Any = None) -> Any:
        """rank 0's obj on every rank."""
        if self.world == 1:
            return obj
        if self.rank == 0:
            for r, c in enumerate(self._peers, 1):
                self._send(c, r, obj)
            return obj
        return self._recv(self._conn, 0)

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
        self._drop_key_file()

    def _drop_key_file(self) -> None:
        if getattr(self, "_key_path", None) and self.rank == 0:
            try:
                os.unlink(self._key_path)
            except OSError:
                pass
            self._key_path = None


def _launch_key(port: int) -> bytes | None:
    """ECGPU_HOSTGROUP_KEY's key, or None: a single-node launch then uses a
    random key passed through a file only this user can read (_key_file)."""
    explicit = os.environ.get("ECGPU_HOSTGROUP_KEY")
    if explicit:
        return hashlib.sha256(explicit.encode()).digest()
    return None


def _private_dir() -> str:
    """This user's 0700 directory for launch keys ($XDG_RUNTIME_DIR or the temp
    dir): another local user can neither read a key nor plant one."""
    import stat
    import tempfile

    base = os.environ.get("XDG_RUNTIME_DIR") or tempfile.gettempdir()
    d = os.path.join(base, f"ecgpu-{os.getuid()}")
    os.makedirs(d, mode=0o700, exist_ok=True)
    st = os.lstat(d)
    if not stat.S_ISDIR(st.st_mode) or st.st_uid != os.getuid() or st.st_mode & 0o077:
        raise PermissionError(f"HostGroup: {d} must be a directory private to this user (owner, mode 0700)")
    return d


def _key_file(port: int) -> str:
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    tag = hashlib.sha256(f"ecgpu-hostgroup|{run}|{port}".encode()).hexdigest()[:24]
    return os.path.join(_private_dir(), f"hostgroup-{tag}.key")


def _write_private(path: str, data: bytes) -> None:
    tmp = f"{path}.{os.getpid()}.tmp"
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
    try:
        os.write(fd, data)
    finally:
        os.close(fd)
    os.replace(tmp, path)  # atomic: a reader sees the old key or the new one, never a part


def _read_private(path: str) -> bytes:
    import stat

    st = os.lstat(path)
    if not stat.S_ISREG(st.st_mode) or st.st_uid != os.getuid() or st.st_mode & 0o077:
        raise PermissionError(f"HostGroup: launch key {path} is not a private file of this user")
    with open(path, "rb") as f:
        return f.read()


def _mac(key: bytes, label: bytes, c0: bytes, c1: bytes, rank: int) -> bytes:
    import hmac

    return hmac.new(key, label + b"|" + c0 + c1 + rank.to_bytes(4, "little"), hashlib.sha256).digest()


def _recv_exact(c, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = c.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("HostGroup: peer closed the connection")
        buf += chunk
    return bytes(buf)


def _enc(o):
    if o is None or isinstance(o, (bool, int, float, str)):
        return o
    if isinstance(o, (bytes, bytearray)):
        return {"$b": bytes(o).hex()}
    if isinstance(o, (list, tuple)):
        return [_enc(x) for x in o]
    if isinstance(o, dict) and all(isinstance(k, str) and not k.startswith("$") for k in o):
        return {k: _enc(v) for k, v in o.items()}
    mod = type(o).__module__
    if mod == "numpy" and type(o).__name__ == "ndarray":  # plain numeric arrays: dtype, shape, bytes
        if o.dtype.kind not in "biuf":
            raise TypeError(f"HostGroup carries numeric arrays only, not dtype {o.dtype}")
        return {"$a": [o.dtype.str, list(o.shape), o.tobytes().hex()]}
    if mod == "numpy" and hasattr(o, "item"):  # numpy scalars
        return _enc(o.item())
    raise TypeError(f"HostGroup carries plain values only, not {type(o).__name__}")


def _dec(o):
    if isinstance(o, list):
        return [_dec(x) for x in o]
    if isinstance(o, dict):
        if set(o) == {"$b"}:
            return bytes.fromhex(o["$b"])
        if set(o) == {"$a"}:
            import numpy as np

            dt, shape, hx = o["$a"]
            dtype = np.dtype(dt)
            if dtype.kind not in "biuf":
                raise ValueError(f"HostGroup: refused array dtype {dt!r}")
            return np.frombuffer(bytes.fromhex(hx), dtype=dtype).reshape(shape).copy()
        return {k: _dec(v) for k, v in o.items()}
    return o


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
              make_id: Callable[[], bytes] | None = None, rccl_at_world1: bool = False,
              timeout_s: float | None = None) -> bytes:
    """Rank 0 makes the RCCL id (make_id, default ecg_comm_unique_id), the
    launcher's group broadcasts it (broadcast(obj) -> rank 0's obj, e.g.
    HostGroup.broadcast), every rank binds its Program's context
    (ecg_comm_init).  make_id is injectable so the CPU tests run the same
    exchange without RCCL.  At world 1 no communicator is made unless
    rccl_at_world1 (a real one-rank RCCL communicator: the RCCL code path on a
    one-GPU box).  timeout_s bounds initialisation and every exchange
    (ecg_comm_set_timeout).  Returns the 128-byte id every rank used."""
    import ctypes

    import ecgpu

    buf = (ctypes.c_uint8 * 128)()
    if world > 1 and broadcast is None:
        raise ValueError("comm_init: world > 1 needs a broadcast(obj) -> rank 0's obj callable "
                         "(e.g. HostGroup.from_env().broadcast)")
    if world > 1:
        ident = None
        if rank == 0:
            ident = make_id() if make_id is not None else unique_id()
        ident = broadcast(ident)
        if not isinstance(ident, (bytes, bytearray)) or len(ident) != 128:
            raise ValueError("comm_init: the broadcast RCCL id must be 128 bytes")
        ctypes.memmove(buf, bytes(ident), 128)
    elif rccl_at_world1:
        ctypes.memmove(buf, make_id() if make_id is not None else unique_id(), 128)
    if prog is None:  # exchange only (CPU tests)
        return bytes(buf)
    L = ecgpu.lib()
    if timeout_s is not None:
        ecgpu._check(L.ecg_comm_set_timeout(prog.handle, int(timeout_s * 1000)), "comm_set_timeout")
    ecgpu._check(L.ecg_comm_init(prog.handle, world, rank, buf if world > 1 or rccl_at_world1 else None),
                 "comm_init")
    return bytes(buf)


def comm_init_host(prog, rank: int, world: int, exchange: Callable[[int, bytes, int], bytes],
                   timeout_s: float | None = None) -> None:
    """Bind prog's context to a host transport (ecg_comm_init_host) instead of
    RCCL: exchange(op, send, nbytes) -> recv bytes, with op XCHG_ALLGATHER
    (send = nbytes, recv = world x nbytes in rank order) or XCHG_ALLTOALL
    (send = world x nbytes, block q to rank q; recv block q from rank q).
    For ranks that share a GPU (RCCL refuses them) and for launchers that
    already hold a group.  A raising exchange fails the call on this rank."""
    import ctypes

    import ecgpu

    def cb(op, send, recv, nbytes, _user):
        try:
            data = ctypes.string_at(send, nbytes * (world if op == ecgpu.XCHG_ALLTOALL else 1))
            out = exchange(op, data, nbytes)
            if len(out) != nbytes * world:
                return 1
            ctypes.memmove(recv, out, len(out))
            return 0
        except Exception as e:  # noqa: BLE001 -- any transport failure is a failed exchange
            import sys
            print(f"ecgpu.dist: host exchange on rank {rank} failed: {type(e).__name__}: {e}", file=sys.stderr)
            return 1

    c_cb = ecgpu.XCHG_CB(cb)
    prog._xchg_cb = c_cb  # the context keeps calling it: keep it alive with the Program
    L = ecgpu.lib()
    if timeout_s is not None:
        ecgpu._check(L.ecg_comm_set_timeout(prog.handle, int(timeout_s * 1000)), "comm_set_timeout")
    ecgpu._check(L.ecg_comm_init_host(prog.handle, world, rank, c_cb, None), "comm_init_host")


TRANSPORTS = {0: "none", 1: "rccl", 2: "host", 3: "failed"}


def comm_info(prog) -> dict:
    """What this rank's communicator reports (ecg_comm_info): for RCCL the
    communicator's own ncclCommCount / ncclCommUserRank / ncclCommCuDevice,
    and the PCI bus id of that device."""
    import ctypes

    import ecgpu

    n, r, d, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    bus = ctypes.create_string_buffer(64)
    ecgpu._check(ecgpu.lib().ecg_comm_info(prog.handle, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d), bus,
                                           len(bus), ctypes.byref(t)), "comm_info")
    return {"count": n.value, "rank": r.value, "device": d.value, "pci_bus_id": bus.value.decode(),
            "transport": TRANSPORTS.get(t.value, str(t.value))}


def last_exchange_us(prog) -> float:
    """Wall time of the last msm_dist's status + partial exchange (us)."""
    import ctypes

    import ecgpu

    us = ctypes.c_double()
    ecgpu._check(ecgpu.lib().ecg_comm_last_exchange(prog.handle, ctypes.byref(us)), "comm_last_exchange")
    return us.value


def comm_record(infos: list) -> dict:
    """rank 0's summary of every rank's comm_info (bench.py's `rccl` field):
    the rank count the communicators hold, their ranks in order, their
    devices by PCI bus id, and whether those devices are distinct."""
    buses = [i["pci_bus_id"] for i in infos]
    return {"transport": sorted({i["transport"] for i in infos}),
            "count": sorted({i["count"] for i in infos}),
            "ranks": [i["rank"] for i in infos],
            "devices": buses,
            "distinct": len(set(buses)) == len(buses)}


class LocalExchange:
    """In-process host transport for `world` ranks driven by threads (one
    context each, e.g. all on one GPU): exchange_for(rank) is the rank's
    comm_init_host callable.  A rank that does not arrive within timeout_s
    breaks the barrier and every waiting rank's exchange fails."""

    def __init__(self, world: int, timeout_s: float = 120.0):
        import threading

        self.world = world
        self._slots: list = [None] * world
        self._barrier = threading.Barrier(world, timeout=timeout_s)

    def exchange_for(self, rank: int) -> Callable[[int, bytes, int], bytes]:
        import ecgpu

        def exchange(op: int, data: bytes, nbytes: int) -> bytes:
            self._slots[rank] = data
            self._barrier.wait()
            if op == ecgpu.XCHG_ALLGATHER:
                out = b"".join(self._slots)
            else:
                out = b"".join(self._slots[q][rank * nbytes:(rank + 1) * nbytes] for q in range(self.world))
            self._barrier.wait()  # nobody overwrites a slot before every rank has read it
            return out

        return exchange


def hostgroup_exchange(group: "HostGroup", piece: int = 256 << 10) -> Callable[[int, bytes, int], bytes]:
    """comm_init_host callable over a HostGroup.  Its frames are capped at
    1 MiB and carry bytes hex-encoded, and rank 0's all-gather reply holds
    every rank's piece, so payloads go in pieces of at most `piece` bytes and
    at most (cap - slack) / (2 x world) -- one all-gather each.  Meant for the
    status records and partial points, and for rehearsal-size all-to-alls, not
    for bulk data."""
    import ecgpu

    piece = max(1, min(piece, (HostGroup._MAX_FRAME - 4096) // (2 * max(group.world, 1))))

    def exchange(op: int, data: bytes, nbytes: int) -> bytes:
        parts = [group.allgather(data[o:o + piece]) for o in range(0, max(len(data), 1), piece)]
        blocks = [b"".join(p[r] for p in parts) for r in range(group.world)]
        if op == ecgpu.XCHG_ALLGATHER:
            return b"".join(blocks)
        r = group.rank
        return b"".join(b[r * nbytes:(r + 1) * nbytes] for b in blocks)

    return exchange


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


def msm_dist(prog, curve, d_bases, d_scalars, n_local: int, maybe_abort=None):
    """This rank's shard + all-gather of [status | partial] + fold -> full
    result on every rank, or the same error on every rank (ecg_msm_dist_ex;
    maybe_abort polled before each device pass, multiexp.rs:140-144)."""
    import numpy as np

    import ecgpu

    cid = ecgpu.CURVE_NAMES.get(curve, -1) if isinstance(curve, str) else int(curve)
    out = np.zeros(3 * ecgpu.CURVE_FQ_LIMBS.get(cid, 12), dtype=np.uint64)
    cb, keep = ecgpu._abort_cb(maybe_abort)
    ecgpu._check(ecgpu.lib().ecg_msm_dist_ex(prog.handle, cid, d_bases.ptr if d_bases is not None else None,
                                             d_scalars.ptr if d_scalars is not None else None, n_local,
                                             ecgpu._ptr(out), cb, None), "msm_dist")
    del keep
    return out


def msm_dist_grid(prog, curve, d_bases, d_scalars, n: int, maybe_abort=None):
    """Grid split (ecg_msm_dist_grid_ex): every rank passes ALL n bases and
    scalars and runs 1/world of the n-term plan's (window x term) grid; the
    [status | partial] records are exchanged and folded as in msm_dist."""
    import numpy as np

    import ecgpu

    cid = ecgpu.CURVE_NAMES.get(curve, -1) if isinstance(curve, str) else int(curve)
    out = np.zeros(3 * ecgpu.CURVE_FQ_LIMBS.get(cid, 12), dtype=np.uint64)
    cb, keep = ecgpu._abort_cb(maybe_abort)
    ecgpu._check(ecgpu.lib().ecg_msm_dist_grid_ex(prog.handle, cid, d_bases.ptr if d_bases is not None else None,
                                                  d_scalars.ptr if d_scalars is not None else None, n,
                                                  ecgpu._ptr(out), cb, None), "msm_dist_grid")
    del keep
    return out


def fft_dist(prog, field, d_local, omega, log_n: int, maybe_abort=None) -> None:
    """One 2^log_n NTT, block-distributed over the communicator (in place);
    statuses exchanged before the first and the last all-to-all."""
    import numpy as np

    import ecgpu

    om = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
    fid = ecgpu.FIELD_NAMES.get(field, -1) if isinstance(field, str) else int(field)
    cb, keep = ecgpu._abort_cb(maybe_abort)
    ecgpu._check(ecgpu.lib().ecg_fft_dist_ex(prog.handle, fid, d_local.ptr if d_local is not None else None,
                                             ecgpu._ptr(om), log_n, cb, None), "fft_dist")
    del keep


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
