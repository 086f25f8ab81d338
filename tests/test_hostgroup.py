"""HostGroup (ecgpu.dist): the N>1 launch's control channel (RCCL id,
barriers, max over ranks).  Checks the wire format carries plain values only,
that rank 0 authenticates peers (challenge + HMAC) and survives bad or
duplicate joiners, and that a missing broadcast is a clear error."""
import os
import socket
import sys
import threading

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
from ecgpu import dist as edist  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_wire_format_plain_values_only():
    vals = [None, True, 3, -2.5, "x", b"\x00\xff" * 64, [1, [2, b"z"]], {"a": 1, "b": [None]},
            np.arange(6, dtype=np.uint64).reshape(2, 3), np.float64(1.5)]
    for v in vals:
        got = edist._dec(edist._enc(v))
        if isinstance(v, np.ndarray):
            assert got.dtype == v.dtype and (got == v).all()
        else:
            assert got == (v.item() if isinstance(v, np.generic) else v)

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    for bad in (Evil(), {1: 2}, {"$b": "00"}, np.array(["s"]), object()):
        with pytest.raises(TypeError):
            edist._enc(bad)
    with pytest.raises(ValueError):
        edist._dec({"$a": ["|O", [1], "00"]})


def _rank(rank, world, port, out, key=None):
    g = edist.HostGroup(rank, world, "127.0.0.1", port, key=key, timeout=30)
    try:
        out[rank] = (g.broadcast(b"id" * 64 if rank == 0 else None), g.allgather(rank * 10), g.max(rank + 0.5))
        g.barrier()
    finally:
        g.close()


def test_hostgroup_rejects_bad_and_duplicate_peers():
    port = _free_port()
    out = {}
    key = b"k" * 32
    t0 = threading.Thread(target=_rank, args=(0, 3, port, out, key))
    t0.start()
    # an intruder with the wrong key, one claiming an out-of-range rank, and a
    # silent connection: each is dropped, rank 0 keeps accepting
    for claim, k in ((1, b"wrong" * 8), (7, key)):
        while True:
            try:
                c = socket.create_connection(("127.0.0.1", port), timeout=5)
                break
            except OSError:
                pass
        ch = edist._recv_exact(c, 32)
        c.sendall(claim.to_bytes(4, "little") + edist._mac(k, ch, claim))
        assert c.recv(2) == b""  # closed without "ok"
        c.close()
    t1 = threading.Thread(target=_rank, args=(1, 3, port, out, key))
    t2 = threading.Thread(target=_rank, args=(2, 3, port, out, key))
    t1.start()
    t2.start()
    for t in (t0, t1, t2):
        t.join(60)
    assert set(out) == {0, 1, 2}
    for r in range(3):
        bid, gathered, mx = out[r]
        assert bid == b"id" * 64 and gathered == [0, 10, 20] and mx == 2.5


def test_hostgroup_duplicate_rank_refused():
    """_admit refuses a correctly authenticated rank that already joined."""
    g = edist.HostGroup(0, 1)
    g.world, g._key, g._timeout = 3, b"d" * 32, 5.0
    for peers, want in (({1: None}, None), ({}, 1)):
        a, b = socket.socketpair()

        def client():
            ch = edist._recv_exact(b, 32)
            b.sendall((1).to_bytes(4, "little") + edist._mac(g._key, ch, 1))

        t = threading.Thread(target=client)
        t.start()
        assert g._admit(a, peers) == want
        t.join(10)
        a.close()
        b.close()


def test_comm_init_needs_broadcast():
    with pytest.raises(ValueError, match="broadcast"):
        edist.comm_init(None, 1, 2, None, make_id=lambda: bytes(128))
    assert edist.comm_init(None, 0, 1) == bytes(128)
