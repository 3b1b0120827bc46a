"""Frame-batch sharding over the GPUs of a node.

Frames are independent, so the hot path has no exchange step: every rank detects on its own
contiguous block of frames with its own fd_ctx (one process per GPU), and no collective touches
the data path. The only collectives are control-plane ones: a barrier and a max-reduce for timing,
and an optional gather of the (small) per-frame feature lists to one rank. They run over whatever
process group the caller initialised (RCCL "nccl" on GPUs, "gloo" on CPU).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [start, end) of `total` frames owned by `rank` (sizes differ by at most 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a float over all ranks (timing); identity without a process group."""
    if dist is None or not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def detect_sharded(frames: np.ndarray, detect: Callable[[np.ndarray], Sequence[np.ndarray]], dist=None,
                   gather: bool = True) -> list[np.ndarray] | None:
    """Run `detect` on this rank's block of `frames` ([B, R, C]); optionally gather all blocks.

    detect(block) returns one (n_i, 2) feature array per frame of the block. With gather=True every
    rank receives the features of all B frames in frame order (an all_gather of small Python objects;
    not on the data path). Without a process group this is a plain call.
    """
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return list(detect(frames))
    rank, world = dist.get_rank(), dist.get_world_size()
    s, e = shard_range(len(frames), rank, world)
    local = [np.asarray(f) for f in detect(frames[s:e])] if e > s else []
    if not gather:
        return local
    parts: list = [None] * world
    dist.all_gather_object(parts, local)
    return [f for part in parts for f in part]
