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
