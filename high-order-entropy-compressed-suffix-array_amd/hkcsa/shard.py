"""Host orchestration of the sharded suffix-array build (see csrc/hk_shard.hip).

The native entry point hkcsa_build_sa_sharded does the whole exchange itself over
RCCL.  This module is the host-driven variant for hosts that run their own
collectives (torch.distributed over RCCL or gloo) and for ranks emulated on one GPU:

    h = dev.shard_histogram(N, r)            # key-prefix histogram of the block (65536 u64)
    g = allreduce_sum(h)                     # collective 1
    c = dev.shard_counts(g, N, r)            # block suffixes below each splitter
    G = allreduce_sum(c)                     # collective 2: N+1 u64 -> exact slice bounds
    dev.shard_build(g, G, N, r)              # independent slice sort + chunk refinement
    shard_doubling(dev, r, allgather)        # repetitive texts only: prefix doubling with the
                                             # ISA rank exchange

Two partition schemes (dev.shard_scheme(), decided by the alphabet): 1 = keyed coarse, the
exact histogram of the top 16 bits of each suffix's keyed sym field (DNA and the other
whole-symbol keyed radixes; collective 2 is then redundant: G follows from g); 0 = the sampled
14-bit partition key.  split_buckets() restates the splitter rule of hk_shard.hip (splitters):
B_r is the first bucket whose prefix count reaches floor(S*r/N), S = the histogram total, except
that the keyed scheme takes the equal-width splitters r * nb / N when N divides nb and none of
their slices holds more than S/N + S/N/50; rank r owns buckets [B_r, B_{r+1}) and its SA slice
is [G[r], G[r+1]).

Prefix doubling across slices.  A slice whose tied groups survive the chunk refinement
(long repeats / runs) stops with its groups pending (hkcsa_shard_status: A tied suffixes
sharing their first h symbols).  Every pending rank then loads a replica of the global ISA
from all ranks' SA slices (a tied suffix's ISA is the slot of its group head, sent as
(position, ISA) pairs), and each round sorts its groups by ISA[p + h] at K = the smallest h
of any pending rank, after which the re-ranked suffixes' pairs are exchanged again.
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np

SH_BUCKETS = 1 << 14
SH_SAMPLE = 64
MAX_ROUNDS = 64


def split_buckets(global_hist, nranks: int, aligned: bool = False) -> list[int]:
    cum = np.concatenate(([0], np.cumsum(np.asarray(global_hist, dtype=np.uint64))))
    tot = int(cum[-1])
    nb = len(cum) - 1
    if aligned and nb % nranks == 0:
        eq = [nb * r // nranks for r in range(nranks + 1)]
        cap = tot // nranks + tot // nranks // 50
        if all(int(cum[eq[r + 1]]) - int(cum[eq[r]]) <= cap for r in range(nranks)):
            return eq
    out = [0]
    for r in range(1, nranks):
        target = (tot * r) // nranks
        out.append(int(np.searchsorted(cum, target, side="left")))
    out.append(len(cum) - 1)
    return out


def slice_bounds(global_below, nranks: int) -> list[tuple[int, int]]:
    g = [int(x) for x in global_below]
    return [(g[r], g[r + 1]) for r in range(nranks)]


def _min_level(status) -> int:
    return min(int(s[3]) for s in status if int(s[2]) > 0)


def shard_doubling(dev, rank: int, allgather: Callable[[np.ndarray], Sequence[np.ndarray]]) -> int:
    """Finish this rank's slice after shard_build (collective: every rank calls it).

    allgather(a) returns the list of every rank's array (arrays may differ in length).
    Returns the number of doubling rounds run (0 when no slice had ties left)."""
    st = allgather(np.array(dev.shard_status(), dtype=np.uint64))
    if sum(int(s[2]) for s in st) == 0:
        return 0
    active = int(st[rank][2]) > 0
    segs = allgather(dev.shard_sa())
    if active:
        for r, seg in enumerate(segs):
            dev.shard_isa_segment(seg, int(st[r][0]))
    pairs = allgather(dev.shard_updates())
    rounds = 0
    while True:
        if rounds >= MAX_ROUNDS:
            raise RuntimeError("sharded prefix doubling did not converge")
        if active:
            for p in pairs:
                dev.shard_apply(p)
        K = _min_level(st)
        dev.shard_round(K)       # an inactive rank's round clears its pairs (nothing is re-sent)
        rounds += 1
        st = allgather(np.array(dev.shard_status(), dtype=np.uint64))
        if sum(int(s[2]) for s in st) == 0:
            return rounds
        pairs = allgather(dev.shard_updates())
        active = int(st[rank][2]) > 0


def emulated_doubling(devs: Sequence) -> int:
    """shard_doubling for N ranks emulated in one process (devs[r] = rank r's handle)."""
    st = [d.shard_status() for d in devs]
    if sum(s[2] for s in st) == 0:
        return 0
    segs = [d.shard_sa() for d in devs]
    for d, s in zip(devs, st):
        if s[2] > 0:
            for r, seg in enumerate(segs):
                d.shard_isa_segment(seg, st[r][0])
    pairs = [d.shard_updates() for d in devs]
    rounds = 0
    while True:
        if rounds >= MAX_ROUNDS:
            raise RuntimeError("sharded prefix doubling did not converge")
        K = _min_level(st)
        for d, s in zip(devs, st):
            if s[2] > 0:
                for p in pairs:
                    d.shard_apply(p)
        for d in devs:
            d.shard_round(K)     # inactive ranks: clears their pairs
        rounds += 1
        st = [d.shard_status() for d in devs]
        if sum(s[2] for s in st) == 0:
            return rounds
        pairs = [d.shard_updates() for d in devs]


def sharded_build(dev, nranks: int, rank: int, allreduce_sum: Callable[[np.ndarray], np.ndarray],
                  allgather: Callable[[np.ndarray], Sequence[np.ndarray]] | None = None):
    """Host-driven sharded SA build; returns this rank's (lo, hi) slice of the SA.

    Without `allgather` a slice whose ties outlast the chunk rounds cannot be finished (the prefix
    doubling needs the rank exchange): that raises instead of returning a slice in tied order."""
    h = dev.shard_histogram(nranks, rank)
    g = allreduce_sum(h)
    c = dev.shard_counts(g, nranks, rank)
    below = allreduce_sum(c)
    dev.shard_build(g, below, nranks, rank)
    if allgather is not None:
        shard_doubling(dev, rank, allgather)
    elif int(dev.shard_status()[2]) > 0:
        raise RuntimeError("sharded_build: this slice needs prefix doubling with the rank exchange; "
                           "pass an allgather")
    return dev.shard_range()
