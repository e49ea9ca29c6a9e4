"""World-size-2 gloo test of the sharded-build orchestration (CPU only).

Each rank runs hkcsa.shard.sharded_build with a CPU stand-in device whose two
phases are the oracle's restatement of the GPU kernels (key-prefix histogram of
the rank's block; slice = its buckets' suffixes in suffix order).  The
collectives are real torch.distributed gloo all-reduce / all-gather, exactly as a
torch host would drive the native two-phase API.  The gathered slices must
concatenate to the oracle suffix array.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


class OracleShardDevice:
    """CPU stand-in for DeviceIndex's shard_* methods (test infrastructure)."""

    def __init__(self, text: np.ndarray):
        from oracle import oracle
        self.o = oracle
        self.t = text
        self.n = len(text)

    def shard_histogram(self, nranks, rank):
        lo, hi = self.n * rank // nranks, self.n * (rank + 1) // nranks
        return self.o.shard_hist(self.t, lo, hi)

    def shard_counts(self, g, nranks, rank):
        from hkcsa.shard import split_buckets
        lo, hi = self.n * rank // nranks, self.n * (rank + 1) // nranks
        return self.o.shard_below(self.t, lo, hi, split_buckets(g, nranks, aligned=self.o.shard_scheme(self.t) > 0))

    def shard_build(self, g, below, nranks, rank):
        from hkcsa.shard import slice_bounds
        self.lo, self.hi = slice_bounds(below, nranks)[rank]
        full = self.o.suffix_array(self.t)  # the oracle's SA restricted to the owned rank range
        self.slice = full[self.lo:self.hi]

    def shard_range(self):
        return self.lo, self.hi

    def shard_status(self):
        return (self.lo, self.hi, 0, 0)   # the oracle slice is final


class DoublingShardDevice(OracleShardDevice):
    """Adds a CPU model of the sharded prefix-doubling steps (hk_sa.hip k_dbl_*, hk_shard.hip):
    shard_build stops with the slice's suffixes grouped only by their first h0 symbols (members of
    a group in scrambled order, as after the chunk refinement), and every round sorts each group by
    ISA[p + h] from the rank's ISA replica, exactly as the GPU rounds do."""

    def __init__(self, text: np.ndarray, h0: int):
        super().__init__(text)
        self.h0 = h0

    def _share(self, a, b, h):
        t, n = self.t, self.n
        if a + h > n or b + h > n:
            return a == b
        return bytes(t[a:a + h]) == bytes(t[b:b + h])

    def shard_build(self, g, below, nranks, rank):
        super().shard_build(g, below, nranks, rank)
        sl = [int(x) for x in self.slice]
        groups, i = [], 0
        while i < len(sl):
            j = i + 1
            while j < len(sl) and self._share(sl[i], sl[j], self.h0):
                j += 1
            groups.append((i, j))
            i = j
        self.sa = list(sl)
        for a, b in groups:          # unspecified order inside a tied group
            self.sa[a:b] = self.sa[a:b][::-1]
        self.groups = [(a, b) for a, b in groups if b - a > 1]
        self.h = self.h0
        self.isa = None
        self.pairs = [(self.sa[j], self.lo + a) for a, b in self.groups for j in range(a, b)]

    def shard_status(self):
        return (self.lo, self.hi, sum(b - a for a, b in self.groups), self.h)

    def shard_sa(self):
        return np.array(self.sa, dtype=np.uint64)

    def shard_isa_segment(self, seg, lo):
        if self.isa is None:
            self.isa = np.zeros(self.n, dtype=np.int64)
        self.isa[np.asarray(seg, dtype=np.int64)] = lo + np.arange(len(seg))

    def shard_updates(self):
        return np.array(self.pairs, dtype=np.uint64).reshape(-1, 2)

    def shard_apply(self, pairs):
        for p, v in np.asarray(pairs, dtype=np.int64).reshape(-1, 2):
            self.isa[p] = v

    def shard_round(self, K):
        n, h = self.n, self.h
        new_groups, self.pairs = [], []
        for a, b in self.groups:
            mem = sorted(self.sa[a:b], key=lambda p: int(self.isa[p + h]) + 1 if p + h < n else 0)
            self.sa[a:b] = mem
            key = [int(self.isa[p + h]) + 1 if p + h < n else 0 for p in mem]
            i = 0
            while i < len(mem):
                j = i + 1
                while j < len(mem) and key[j] == key[i]:
                    j += 1
                self.pairs += [(mem[k], self.lo + a + i) for k in range(i, j)]
                if j - i > 1:
                    new_groups.append((a + i, a + j))
                i = j
        self.groups = new_groups
        self.h += K
        self.slice = np.array(self.sa, dtype=np.uint64)


def _worker(rank, world, port, n, q, kind="iid"):
    for p in (PKG, ROOT):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from hkcsa.shard import sharded_build
    from dist_helpers import torch_allgather, torch_allreduce_sum
    from oracle import oracle
    if kind == "iid":
        text = oracle.synth_text(n, b"ACGT", seed=21)
        dev = OracleShardDevice(text)
        lo, hi = sharded_build(dev, world, rank, torch_allreduce_sum())
    else:
        text = np.frombuffer((b"abcab" * n)[:n - 1] + b"$", dtype=np.uint8) if kind == "periodic" else \
            np.frombuffer(b"a" * (n - 1) + b"$", dtype=np.uint8)
        dev = DoublingShardDevice(text, h0=3)
        lo, hi = sharded_build(dev, world, rank, torch_allreduce_sum(), torch_allgather())
        assert dev.shard_status()[2] == 0
    bounds = [None] * world
    dist.all_gather_object(bounds, (lo, hi))
    parts = [None] * world
    dist.all_gather_object(parts, dev.slice.tolist())
    if rank == 0:
        full = oracle.suffix_array(text).tolist()
        cat = [x for p in parts for x in p]
        q.put((bounds, cat == full, len(cat), n))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_build_without_allgather_refuses_tied_slice():
    """A slice left tied after the chunk rounds needs the rank exchange: sharded_build without an
    allgather raises instead of returning the slice in tied order."""
    from hkcsa.shard import sharded_build
    from oracle import oracle  # noqa: F401 (stand-in device uses it)
    text = np.frombuffer(b"a" * 400 + b"$", dtype=np.uint8)
    dev = DoublingShardDevice(text, h0=3)
    with pytest.raises(RuntimeError, match="allgather"):
        sharded_build(dev, 1, 0, lambda h: h)


@pytest.mark.parametrize("world,kind,n", [(2, "iid", 30001), (2, "periodic", 3001), (3, "run", 1501)])
def test_gloo_sharded_orchestration(world, kind, n):
    """iid: the three collectives of the build; periodic / run: slices left tied after the chunk
    rounds finish by prefix doubling with the ISA rank exchange (hkcsa.shard.shard_doubling)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    bounds, ok, m, nn = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok and m == nn
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    assert all(b[1] == c[0] for b, c in zip(bounds, bounds[1:]))
