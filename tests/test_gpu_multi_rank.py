"""GPU: the frame-sharded N>1 path with the real detector on the device.

Two or three ranks (gloo control plane, all on cuda:0 of the one-GPU box) each run fd_points_detect
on their block of the batch (feature_detector_amd/shard.py, as bench.py shards frames); the gathered
features must equal the oracle's for every frame. This is the GPU counterpart of
tests/test_multi_rank.py, whose per-rank detector is the CPU oracle.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import feature_detector_amd as fd
        from feature_detector_amd.shard import detect_sharded, shard_range

        def detect(block):
            res = fd.detect_points("harris", np.ascontiguousarray(block), need=50, min_feature_distance=20,
                                   min_valid_response=30.0)
            return [res.features(b) for b in range(len(block))]

        feats = detect_sharded(frames, detect, dist)
        q.put((rank, [f.tolist() for f in feats], shard_range(len(frames), rank, world)))
    except Exception as e:  # reported to the parent instead of a silent hang
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ranks_match_oracle(oracle, world):
    import torch.multiprocessing as mp

    frames = np.stack([oracle.make_frame("noise" if i % 2 else "checker", 70 + i, 120, 160) for i in range(7)])
    expected = [oracle.detect(0, f, 20, 30.0, 50, sort_mode=0)[0].tolist() for f in frames]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = [q.get(timeout=100) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    spans = {}
    for rank, feats, span in results:
        assert span is not None, feats
        assert feats == expected
        spans[rank] = span
    assert sorted(spans) == list(range(world))
    for p in procs:
        assert p.exitcode == 0


def test_two_contexts_on_two_streams_match_oracle(oracle):
    """The serving pipeline bench.py reports as headline_pipelined: consecutive frames alternate
    between two contexts, each on its own stream, with no synchronisation between the streams."""
    import torch

    import feature_detector_amd as fd

    dev = torch.device("cuda", 0)
    frames = [oracle.make_frame("noise" if i % 2 else "checker", 300 + i, 240, 320) for i in range(8)]
    ctxs = [fd.Context(0), fd.Context(0)]
    streams = [torch.cuda.Stream(device=dev) for _ in ctxs]
    dframes = [torch.from_numpy(f[None]).to(dev) for f in frames]
    torch.cuda.synchronize()
    outs = []
    for i, f in enumerate(dframes):
        k = i % 2
        with torch.cuda.stream(streams[k]):
            xy = torch.empty((1, 51, 2), dtype=torch.float32, device=dev)
            cnt = torch.empty((1,), dtype=torch.int32, device=dev)
            fd.detect_points("harris", f, need=50, min_feature_distance=20, min_valid_response=30.0,
                             out=(xy, cnt), ctx=ctxs[k])
            outs.append((xy, cnt))
    torch.cuda.synchronize()
    for f, (xy, cnt) in zip(frames, outs):
        exp = oracle.detect(0, f, 20, 30.0, 50, sort_mode=0)[0]
        np.testing.assert_array_equal(xy[0, : int(cnt[0])].cpu().numpy(), exp)
    for c in ctxs:
        c.close()
