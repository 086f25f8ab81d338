"""CPU tests of the host-side prep mirror: DensityTracker semantics
(ec-gpu-proxy/src/multiexp_cpu.rs:117-207) and the bitmap the device path
consumes (bitvec<usize, Lsb0>)."""
import numpy as np

import ecgpu


def test_density_tracker_semantics():
    d = ecgpu.DensityTracker.new()
    for _ in range(5):
        d.add_element()
    d.inc(1)
    d.inc(3)
    d.inc(3)  # idempotent (multiexp_cpu.rs:149-154)
    assert d.get_total_density() == 2 and d.get_query_size() == 5
    # extend as an input density: other's first bit coalesces with ours
    o = ecgpu.DensityTracker([True, False, True])
    d2 = ecgpu.DensityTracker([True, False])
    d2.extend(o, True)
    assert d2.bv == [True, False, False, True] and d2.get_total_density() == 2
    d3 = ecgpu.DensityTracker([False, True])
    d3.extend(o, True)
    assert d3.bv == [True, True, False, True] and d3.get_total_density() == 3
    d4 = ecgpu.DensityTracker([False])
    d4.extend(o, False)
    assert d4.bv == [False, True, False, True] and d4.get_total_density() == 2
    e = ecgpu.DensityTracker()
    e.extend(o, True)
    assert e.bv == o.bv and e.total_density == 2


def test_density_words_lsb0_and_generate_exps():
    rng = np.random.default_rng(3)
    bits = rng.random(200) < 0.4
    d = ecgpu.DensityTracker(bits)
    w = d.words()
    assert w.dtype == np.uint64 and w.shape == (4,)
    for i in range(200):
        assert bool((int(w[i // 64]) >> (i % 64)) & 1) == bool(bits[i])
    assert int(w[3]) >> (200 - 192) == 0  # padding bits clear
    exps = np.arange(200 * 4, dtype=np.uint64).reshape(200, 4)
    assert (d.generate_exps(exps) == exps[bits]).all()
    assert ecgpu.FullDensity().generate_exps(exps) is exps


# Restated property tests of the reference (multiexp_cpu.rs:422-578); the
# reference draws from a seeded XorShiftRng, here a seeded numpy generator.
def test_extend_density_regular():
    """test_extend_density_regular (multiexp_cpu.rs:422-467): trackers built in
    k-sized pieces and extended (not as input densities) equal the tracker
    built in one go."""
    rng = np.random.default_rng(0x5962BE5D)
    for k in (2, 4, 8):
        for j in (10, 20, 50):
            count = k * j
            full = ecgpu.DensityTracker.new()
            parts = []
            for i in range(count):
                if i % k == 0:
                    parts.append(ecgpu.DensityTracker.new())
                index = i // k
                if rng.random() < 0.5:
                    full.add_element()
                    parts[index].add_element()
                if parts[index].bv:
                    idx = int(rng.integers(0, len(parts[index].bv)))
                    offset = sum(len(t.bv) for t in parts[:index])
                    full.inc(offset + idx)
                    parts[index].inc(idx)
            combined = ecgpu.DensityTracker.new()
            for t in parts:
                combined.extend(t, False)
            assert combined == full, (k, j)


def test_extend_density_input():
    """test_extend_density_input (multiexp_cpu.rs:469-577): every pairing of
    empty / first-bit-unset / first-bit-set trackers extended as input
    densities (the shared ONE input coalesces)."""
    rng = np.random.default_rng(0x763D318D)
    max_bits = max_density = 10

    def empty():
        return ecgpu.DensityTracker.new()

    def unset():
        dt = ecgpu.DensityTracker.new()
        dt.add_element()
        n = int(rng.integers(1, max_bits))
        target = int(rng.integers(0, max_density))
        for _ in range(1, n):
            dt.add_element()
        for _ in range(target):
            if n > 1:
                dt.inc(int(rng.integers(1, n)))
        assert not dt.bv[0] and len(dt.bv) == n
        return dt

    def set_():
        dt = unset()
        dt.inc(0)
        return dt

    for _ in range(10):
        e1 = empty()
        e1.extend(empty(), True)
        assert e1 == empty()
        for make in (unset, set_):
            e1, x = empty(), make()
            e1.extend(x.clone(), True)
            assert e1 == x
            x = make()
            x2 = x.clone()
            x.extend(empty(), True)
            assert x == x2
        u1, u2 = unset(), unset()
        tot = u1.total_density + u2.total_density
        u1.extend(u2, True)
        assert u1.total_density == tot and not u1.bv[0]
        u1, s1 = unset(), set_()
        tot = u1.total_density + s1.total_density
        u1.extend(s1, True)
        assert u1.total_density == tot and u1.bv[0]
        s1, u1 = set_(), unset()
        tot = s1.total_density + u1.total_density
        s1.extend(u1, True)
        assert s1.total_density == tot and s1.bv[0]
        s1, s2 = set_(), set_()
        tot = s1.total_density + s2.total_density - 1
        s1.extend(s2, True)
        assert s1.total_density == tot and s1.bv[0]
