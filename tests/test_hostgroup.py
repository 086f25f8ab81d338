"""HostGroup (ecgpu.dist): the N>1 launch's control channel (RCCL id,
barriers, max over ranks).  Checks the wire format carries plain values only,
that the handshake is mutual (rank 0 authenticates peers and proves the key
back, so an impostor rank 0 is refused), that every frame is authenticated
(a tampered or replayed frame is refused), that rank 0 survives bad or
duplicate joiners, that a multi-node launch without a key fails closed, and
that a missing broadcast is a clear error."""
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
        c1 = os.urandom(32)
        c.sendall(claim.to_bytes(4, "little") + c1 + edist._mac(k, b"join", ch, c1, claim))
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
            c1 = os.urandom(32)
            b.sendall((1).to_bytes(4, "little") + c1 + edist._mac(g._key, b"join", ch, c1, 1))

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


def test_peer_refuses_impostor_rank0():
    """A process that holds the port but not the key cannot pose as rank 0:
    it cannot produce the accept proof, so the joining rank refuses it."""
    port = _free_port()
    ls = socket.socket()
    ls.bind(("127.0.0.1", port))
    ls.listen(1)

    def impostor():
        c, _ = ls.accept()
        c.sendall(os.urandom(32))
        edist._recv_exact(c, 68)
        c.sendall(b"ok" + os.urandom(32))  # no key: a guessed proof
        c.close()

    t = threading.Thread(target=impostor)
    t.start()
    with pytest.raises(ConnectionError, match="prove"):
        edist.HostGroup(1, 2, "127.0.0.1", port, key=b"k" * 32, timeout=10)
    t.join(10)
    ls.close()


def test_frames_are_authenticated():
    """Frames after the handshake carry a session MAC with a sequence number:
    a flipped byte, or a frame replayed, is refused."""
    port = _free_port()
    key = b"f" * 32
    holder = {}

    def r0():
        holder[0] = edist.HostGroup(0, 2, "127.0.0.1", port, key=key, timeout=20)

    t = threading.Thread(target=r0)
    t.start()
    g1 = edist.HostGroup(1, 2, "127.0.0.1", port, key=key, timeout=20)
    t.join(20)
    g0 = holder[0]
    try:
        # a genuine frame goes through
        g1._send(g1._conn, 0, {"v": 1})
        assert g0._recv(g0._peers[0], 1) == {"v": 1}
        # capture the next frame on the wire, then deliver it tampered
        a, b = socket.socketpair()
        g1._send(a, 0, [7, 8])
        raw = edist._recv_exact(b, 8 + len(b"[7,8]") + 32)
        tampered = raw[:8] + b"[7,9]" + raw[8 + 5:]
        c, d = socket.socketpair()
        c.sendall(tampered)
        with pytest.raises(ConnectionError, match="authentication"):
            g0._recv(d, 1)
        # the genuine frame, delivered twice: the replay fails (sequence number)
        e, f = socket.socketpair()
        e.sendall(raw + raw)
        # (the refused tampered copy consumed no sequence number)
        assert g0._recv(f, 1) == [7, 8]
        with pytest.raises(ConnectionError, match="authentication"):
            g0._recv(f, 1)
        for sck in (a, b, c, d, e, f):
            sck.close()
    finally:
        g1.close()
        g0.close()


def test_multinode_launch_without_key_fails_closed(monkeypatch):
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("MASTER_ADDR", "10.0.0.1")
    monkeypatch.delenv("ECGPU_HOSTGROUP_KEY", raising=False)
    with pytest.raises(PermissionError, match="ECGPU_HOSTGROUP_KEY"):
        edist.HostGroup.from_env()


def test_hostgroup_exchange_allgather_alltoall_in_pieces():
    """ecgpu.dist.hostgroup_exchange (the host transport of ecg_comm_init_host
    over a HostGroup): all-gather and all-to-all semantics, with payloads cut
    into pieces below the frame cap."""
    import ecgpu

    port = _free_port()
    world, nb = 3, 1000
    out = {}

    def rank(r):
        g = edist.HostGroup(r, world, "127.0.0.1", port, key=b"x" * 32, timeout=30)
        try:
            ex = edist.hostgroup_exchange(g, piece=256)  # tiny pieces: many rounds
            mine = bytes([r]) * nb
            ag = ex(ecgpu.XCHG_ALLGATHER, mine, nb)
            send = b"".join(bytes([16 * r + q]) * nb for q in range(world))  # block q -> rank q
            a2a = ex(ecgpu.XCHG_ALLTOALL, send, nb)
            out[r] = (ag, a2a)
        finally:
            g.close()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    for r in range(world):
        ag, a2a = out[r]
        assert ag == b"".join(bytes([q]) * nb for q in range(world))
        assert a2a == b"".join(bytes([16 * q + r]) * nb for q in range(world))


def test_hostgroup_exchange_default_pieces_fit_the_frame_cap():
    """The default piece size shrinks with the world so rank 0's all-gather
    reply (every rank's piece, hex-encoded) stays under the frame cap: a
    multi-MiB all-to-all at world 4 goes through."""
    import ecgpu

    port = _free_port()
    world, nb = 4, 600 << 10
    out = {}

    def rank(r):
        g = edist.HostGroup(r, world, "127.0.0.1", port, key=b"y" * 32, timeout=60)
        try:
            ex = edist.hostgroup_exchange(g)
            send = b"".join(bytes([16 * r + q]) * nb for q in range(world))
            out[r] = ex(ecgpu.XCHG_ALLTOALL, send, nb)
        finally:
            g.close()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    for r in range(world):
        assert out[r] == b"".join(bytes([16 * q + r]) * nb for q in range(world))


def test_single_node_key_is_random_and_private(monkeypatch, tmp_path):
    """without ECGPU_HOSTGROUP_KEY a single-node launch's key is
    random (not derivable from the public run id and port), passes through a
    0600 file in a 0700 per-user directory, and is removed once every rank
    joined; a key file another user could write is refused."""
    import stat

    monkeypatch.delenv("ECGPU_HOSTGROUP_KEY", raising=False)
    monkeypatch.setenv("XDG_RUNTIME_DIR", str(tmp_path))
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    port = _free_port()
    path = edist._key_file(port)
    d = os.path.dirname(path)
    assert stat.S_IMODE(os.stat(d).st_mode) == 0o700
    out, keys = {}, {}

    def rank(r):
        g = edist.HostGroup(r, 3, "127.0.0.1", port, timeout=60)
        keys[r] = g._key
        out[r] = g.allgather(r * 7)
        g.close()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert out == {0: [0, 7, 14], 1: [0, 7, 14], 2: [0, 7, 14]}
    assert keys[0] == keys[1] == keys[2] and len(keys[0]) == 32
    assert keys[0] != edist.hashlib.sha256(f"ecgpu-hostgroup|none|{port}".encode()).digest()
    assert not os.path.exists(path)  # removed after the handshake
    # a key file that is group/other-writable is not trusted
    edist._write_private(path, b"x" * 32)
    os.chmod(path, 0o644)
    with pytest.raises(PermissionError, match="private"):
        edist._read_private(path)
    os.unlink(path)
    # a shared (not 0700) key directory is refused
    os.chmod(d, 0o755)
    with pytest.raises(PermissionError, match="0700"):
        edist._private_dir()
    os.chmod(d, 0o700)
