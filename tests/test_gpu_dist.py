"""Multi-process sharded build on the GPU: world-size 2 / 3 processes (gloo collectives, all ranks on
the one MI355X of the box), each rank a real DeviceIndex running the native slice kernels through
hkcsa.shard.sharded_build — the host-driven phase API (hkcsa_shard_histogram / _counts / _build /
_status / _isa_segment / _updates / _apply / _round) exactly as a torch host drives it, with the
coarse-histogram all-reduce, the slice-count all-reduce and, for repetitive text, the prefix-doubling
rank exchange across processes.  Every rank checks its SA and BWT rows against the oracle
(reference: csa/suffix_array.py:131-134, csa/bwt.py:3-13); rank 0 checks that the slices tile [0, n).
The RCCL path of hkcsa_build_sa_sharded needs one GPU per rank, which a one-GPU box does not have.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _texts(kind: str, n: int) -> np.ndarray:
    from oracle import oracle
    if kind == "dna":
        return oracle.synth_text(n, b"ACGT", seed=31)
    if kind == "bytes":
        return oracle.synth_text(n, bytes(range(1, 256)), seed=32)
    if kind == "printable":
        return oracle.synth_text(n, bytes(range(32, 127)), seed=33)
    if kind == "periodic":
        return np.frombuffer((b"abcab" * n)[:n - 1] + b"$", dtype=np.uint8)
    raise ValueError(kind)


def _worker(rank, world, port, kind, n, q):
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg, bounds = False, "", None
    try:
        from hkcsa import DeviceIndex
        from hkcsa.shard import sharded_build
        from dist_helpers import torch_allgather, torch_allreduce_sum
        from oracle import oracle
        text = _texts(kind, n)
        dev = DeviceIndex.from_bytes(text, device=0)
        lo, hi = sharded_build(dev, world, rank, torch_allreduce_sum(), torch_allgather())
        assert dev.shard_status()[2] == 0, "slice left tied"
        ref = oracle.suffix_array(text)
        sa, bwt = dev.shard_sa(), dev.shard_bwt()
        ok = bool(np.array_equal(sa, ref[lo:hi]) and np.array_equal(bwt, oracle.bwt(text, ref)[lo:hi]))
        msg = "" if ok else f"rank {rank}: slice [{lo}, {hi}) differs from the oracle"
        bounds = (int(lo), int(hi))
        dev.close()
    except Exception as e:  # reported to the parent, which fails the test
        msg = f"rank {rank}: {type(e).__name__}: {e}"
    allb = [None] * world
    dist.all_gather_object(allb, bounds)
    if rank == 0:
        q.put((allb, msg))
    else:
        q.put((None, msg))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,kind,n", [(2, "dna", 1_000_001), (3, "bytes", 400_001),
                                          (2, "printable", 300_001), (2, "periodic", 30_001)])
def test_gloo_native_slices(world, kind, n):
    """dna / bytes: keyed coarse scheme (exact 16-bit histogram, fused selection); printable: the
    partition-key scheme; periodic: slices tied after the chunk rounds finish by prefix doubling with
    the ISA rank exchange between processes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    msgs = [m for _, m in results if m]
    assert not msgs, msgs
    bounds = next(b for b, _ in results if b is not None)
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    assert all(b[1] == c[0] for b, c in zip(bounds, bounds[1:]))
