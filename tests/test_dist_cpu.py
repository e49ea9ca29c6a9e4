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
        return self.o.shard_below(self.t, lo, hi, split_buckets(g, nranks))

    def shard_build(self, g, below, nranks, rank):
        from hkcsa.shard import slice_bounds
        self.lo, self.hi = slice_bounds(below, nranks)[rank]
        full = self.o.suffix_array(self.t)  # the oracle's SA restricted to the owned rank range
        self.slice = full[self.lo:self.hi]

    def shard_range(self):
        return self.lo, self.hi


def _worker(rank, world, port, n, q):
    for p in (PKG, ROOT):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from hkcsa.shard import sharded_build, torch_allreduce_sum
    from oracle import oracle
    text = oracle.synth_text(n, b"ACGT", seed=21)
    dev = OracleShardDevice(text)
    lo, hi = sharded_build(dev, world, rank, torch_allreduce_sum())
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


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_orchestration(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n = 30001
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    bounds, ok, m, nn = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok and m == nn
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    assert all(b[1] == c[0] for b, c in zip(bounds, bounds[1:]))
