"""Host orchestration of the sharded suffix-array build (see csrc/hk_shard.hip).

The native entry point hkcsa_build_sa_sharded does the whole exchange itself over
RCCL.  This module is the three-phase variant for hosts that run their own
collectives (torch.distributed over RCCL or gloo):

    h = dev.shard_histogram(N, r)            # sampled 14-bit key-prefix histogram of the block
    g = allreduce_sum(h)                     # collective 1: 16384 u64
    c = dev.shard_counts(g, N, r)            # block suffixes below each splitter
    G = allreduce_sum(c)                     # collective 2: N+1 u64 -> exact slice bounds
    dev.shard_build(g, G, N, r)              # independent slice sort + refinement

split_buckets() restates the splitter rule of hk_shard.hip (splitters): B_r is the first
bucket whose sampled prefix count reaches floor(S*r/N), S = the sample total; rank r
owns buckets [B_r, B_{r+1}) and its SA slice is [G[r], G[r+1]).
"""
from __future__ import annotations

from typing import Callable

import numpy as np

SH_BUCKETS = 1 << 14
SH_SAMPLE = 16


def split_buckets(global_hist, nranks: int) -> list[int]:
    cum = np.concatenate(([0], np.cumsum(np.asarray(global_hist, dtype=np.uint64))))
    tot = int(cum[-1])
    out = [0]
    for r in range(1, nranks):
        target = (tot * r) // nranks
        out.append(int(np.searchsorted(cum, target, side="left")))
    out.append(len(cum) - 1)
    return out


def slice_bounds(global_below, nranks: int) -> list[tuple[int, int]]:
    g = [int(x) for x in global_below]
    return [(g[r], g[r + 1]) for r in range(nranks)]


def sharded_build(dev, nranks: int, rank: int, allreduce_sum: Callable[[np.ndarray], np.ndarray]):
    """Three-phase sharded SA build; returns this rank's (lo, hi) slice of the SA."""
    h = dev.shard_histogram(nranks, rank)
    g = allreduce_sum(h)
    c = dev.shard_counts(g, nranks, rank)
    below = allreduce_sum(c)
    dev.shard_build(g, below, nranks, rank)
    return dev.shard_range()


def torch_allreduce_sum(group=None) -> Callable[[np.ndarray], np.ndarray]:
    import torch
    import torch.distributed as dist

    def f(h: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.asarray(h, dtype=np.int64).copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t.numpy().astype(np.uint64)
    return f
