"""Host orchestration of the sharded suffix-array build (see csrc/hk_shard.hip).

The native entry point hkcsa_build_sa_sharded does the whole exchange itself over
RCCL.  This module is the two-phase variant for hosts that run their own
collectives (torch.distributed over RCCL or gloo):

    h = dev.shard_histogram(N, r)            # this rank's 14-bit key-prefix histogram
    g = allreduce_sum(h)                     # one collective, 16384 u64
    dev.shard_build(g, N, r)                 # independent slice sort + refinement

slice_bounds() restates the splitter rule of hk_shard.hip (shard_build_t): rank r
owns buckets [B_r, B_{r+1}) where B_r is the first bucket whose prefix count
reaches floor(n*r/N); its slice of the final SA is [cum[B_r], cum[B_{r+1})).
"""
from __future__ import annotations

from typing import Callable

import numpy as np

SH_BUCKETS = 1 << 14


def split_buckets(global_hist, n: int, nranks: int) -> list[int]:
    cum = np.concatenate(([0], np.cumsum(np.asarray(global_hist, dtype=np.uint64))))
    if int(cum[-1]) != n:
        raise ValueError("histogram does not sum to n")
    out = [0]
    for r in range(1, nranks):
        target = (n * r) // nranks
        out.append(int(np.searchsorted(cum, target, side="left")))
    out.append(len(cum) - 1)
    return out


def slice_bounds(global_hist, n: int, nranks: int) -> list[tuple[int, int]]:
    cum = np.concatenate(([0], np.cumsum(np.asarray(global_hist, dtype=np.uint64))))
    b = split_buckets(global_hist, n, nranks)
    return [(int(cum[b[r]]), int(cum[b[r + 1]])) for r in range(nranks)]


def sharded_build(dev, nranks: int, rank: int, allreduce_sum: Callable[[np.ndarray], np.ndarray]):
    """Two-phase sharded SA build; returns this rank's (lo, hi) slice of the SA."""
    h = dev.shard_histogram(nranks, rank)
    g = allreduce_sum(h)
    dev.shard_build(g, nranks, rank)
    return dev.shard_range()


def torch_allreduce_sum(group=None) -> Callable[[np.ndarray], np.ndarray]:
    import torch
    import torch.distributed as dist

    def f(h: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.asarray(h, dtype=np.int64).copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t.numpy().astype(np.uint64)
    return f
