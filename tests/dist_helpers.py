"""Host collectives over torch.distributed (gloo / RCCL host path) for the host-driven sharded build
(hkcsa.shard.sharded_build takes any allreduce / allgather callables; the product package itself does
not import torch).  Test infrastructure."""
from __future__ import annotations

from typing import Callable

import numpy as np


def torch_allreduce_sum(group=None) -> Callable[[np.ndarray], np.ndarray]:
    import torch
    import torch.distributed as dist

    def f(h: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.asarray(h, dtype=np.int64).copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t.numpy().astype(np.uint64)
    return f


def torch_allgather(group=None) -> Callable[[np.ndarray], list[np.ndarray]]:
    """Variable-length all-gather of numpy arrays over torch.distributed (gloo / RCCL host path)."""
    import torch.distributed as dist

    def f(a: np.ndarray) -> list[np.ndarray]:
        out = [None] * dist.get_world_size(group)
        dist.all_gather_object(out, np.asarray(a), group=group)
        return out
    return f
