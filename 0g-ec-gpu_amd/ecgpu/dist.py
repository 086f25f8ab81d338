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
reduction op -- and folded on the device (ecg_point_sum_dev).  FFT: whole
transforms are assigned round-robin-by-chunk; nothing is exchanged.

The compute and fold callables are injected so the same orchestration runs
on the GPU (HIP kernels, backend "nccl") and in the CPU multi-process tests
(backend "gloo").
"""
from __future__ import annotations

from typing import Callable, Sequence


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
