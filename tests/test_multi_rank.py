"""CPU: the N>1 (frame-sharded) path with a world-size-2 gloo process group.

Each rank detects on its own block of a batch and the blocks are gathered in frame order; the
result must equal the unsharded result for every frame. The per-rank detector here is the CPU
oracle (test-only stand-in for the per-GPU fd_ctx, which needs a GPU); the sharding and gathering
code is the package's own (feature_detector_amd/shard.py), as used by bench.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from feature_detector_amd.shard import detect_sharded, max_over_ranks, shard_range
        from oracle import oracle as O

        def detect(block):
            return [O.detect(0, f, 20, 30.0, 50, sort_mode=1)[0] for f in block]

        feats = detect_sharded(frames, detect, dist)
        t = max_over_ranks(float(rank + 1), dist)
        q.put((rank, [f.tolist() for f in feats], t, shard_range(len(frames), rank, world)))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from feature_detector_amd.shard import shard_range

    for total in (0, 1, 7, 256):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_matches_unsharded(oracle):
    frames = np.stack([oracle.make_frame("noise" if i % 2 else "checker", 50 + i, 120, 160) for i in range(5)])
    expected = [oracle.detect(0, f, 20, 30.0, 50, sort_mode=1)[0].tolist() for f in frames]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spans = {}
    for rank, feats, tmax, span in results:
        assert feats == expected  # every rank holds all frames' features, in frame order
        assert tmax == 2.0  # max over ranks
        spans[rank] = span
    assert spans == {0: (0, 3), 1: (3, 5)}
