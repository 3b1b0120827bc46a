"""GPU: equal responses in the greedy scan (SelectGoodFeatures, feature_point_detector.cpp:58-60).

The reference sorts its raster-ordered candidates with an unstable std::sort, so the order of equal
responses is whatever libstdc++'s introsort leaves. k_select flags every frame whose scanned prefix
meets two equal responses (FD_FRAME_TIES); in the default "reference" tie order those frames are
re-selected in std::sort's permutation and must equal the oracle's std::sort order (sort_mode 0),
while "raster" keeps (response desc, raster asc) = the oracle's stable order (sort_mode 1). On the
constructed tie frames the two orders give different feature lists, so both paths are exercised.
"""
import numpy as np
import pytest

from conftest import make_tie_frame

pytestmark = pytest.mark.gpu

THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}
KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2}


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


@pytest.fixture(autouse=True, params=["auto", "wide", "narrow"])
def ref_wide(request, monkeypatch):
    """k_select_reference's multi-workgroup prelude (push order and the first partition levels of large
    frames): by frame size (>= 1 Mpx, "auto"), forced on or forced off (FD_REF_WIDE)."""
    if request.param != "auto":
        monkeypatch.setenv("FD_DEBUG_AB", "1")  # (the library reads A/B switches only with it)
        monkeypatch.setenv("FD_REF_WIDE", "1" if request.param == "wide" else "0")
    return request.param


def _both(fd, oracle, name, frames, need, dist, prior=None):
    ref = fd.detect_points(name, frames, need, dist, THR[name], prior=prior)
    ras = fd.detect_points(name, frames, need, dist, THR[name], prior=prior, ties="raster")
    flags = ref.frame_flags()
    # device frames and outputs: no host fallback behind the GPU emulation (FRAME_UNRESOLVED would raise)
    import torch

    dev = fd.detect_points(name, torch.from_numpy(np.ascontiguousarray(frames)).cuda(), need, dist, THR[name],
                           prior=prior, ties="reference")
    torch.cuda.synchronize()
    dev.check()
    for b in range(frames.shape[0]):
        np.testing.assert_array_equal(dev.features(b), ref.features(b), err_msg=f"{name} frame {b} device path")
        p = None if prior is None else prior[b]
        e0 = oracle.detect(KIND[name], frames[b], dist, THR[name], need, p, sort_mode=0)[0]
        e1 = oracle.detect(KIND[name], frames[b], dist, THR[name], need, p, sort_mode=1)[0]
        np.testing.assert_array_equal(ref.features(b), e0, err_msg=f"{name} frame {b} reference order")
        np.testing.assert_array_equal(ras.features(b), e1, err_msg=f"{name} frame {b} raster order")
        if not np.array_equal(e0, e1):
            assert flags[b] & fd.points.FRAME_TIES and flags[b] & fd.points.FRAME_RESOLVED
    return ref, ras


@pytest.mark.parametrize("name", ["harris", "shi_tomasi"])
def test_tie_frame_orders_differ_and_match_oracle(fd, oracle, name):
    img = make_tie_frame(oracle)
    e0 = oracle.detect(KIND[name], img, 20, THR[name], 200, sort_mode=0)[0]
    e1 = oracle.detect(KIND[name], img, 20, THR[name], 200, sort_mode=1)[0]
    assert not np.array_equal(e0, e1), "the constructed frame must separate the two orders"
    ref, ras = _both(fd, oracle, name, img[None], 200, 20)
    assert not np.array_equal(ref.features(0), ras.features(0))
    assert ras.frame_flags()[0] & fd.points.FRAME_TIES
    assert not ras.frame_flags()[0] & fd.points.FRAME_RESOLVED


def test_tie_frames_in_mixed_batch(fd, oracle):
    frames = np.stack([make_tie_frame(oracle, seed=5), oracle.make_frame("noise", 6, 480, 640),
                       make_tie_frame(oracle, seed=7, copies=(5, 9)), oracle.make_frame("checker", 8, 480, 640)])
    for name in ("harris", "shi_tomasi", "fast"):
        _both(fd, oracle, name, frames, 200, 20)


@pytest.mark.parametrize("dist,need", [(0, 60), (2, 400), (20, 30), (20, 100000)])
def test_tie_frame_selection_regimes(fd, oracle, dist, need):
    # d = 0 (no grid), d = 2 at 1080p (global occupancy grid), a need reached inside the tie run,
    # and a need never reached (every candidate visited)
    rows, cols = (1080, 1920) if dist == 2 else (480, 640)
    img = make_tie_frame(oracle, rows, cols, copies=(9, 12))
    _both(fd, oracle, "harris", img[None], need, dist)


def test_tie_frame_with_priors(fd, oracle):
    img = make_tie_frame(oracle)
    prior = [np.array([(x, y) for x in range(30, 640, 97) for y in range(40, 480, 113)], np.float32)]
    _both(fd, oracle, "harris", img[None], 200, 20, prior)


def test_device_frames_reference_order(fd, oracle):
    torch = pytest.importorskip("torch")
    host = np.stack([make_tie_frame(oracle, seed=s) for s in (1, 2)])
    dev = torch.from_numpy(host).cuda()
    res = fd.detect_points("shi_tomasi", dev, 200, 20, 40.0, ties="reference")
    torch.cuda.synchronize()
    for b in range(2):
        e0 = oracle.detect(1, host[b], 20, 40.0, 200, sort_mode=0)[0]
        np.testing.assert_array_equal(res.features(b), e0)
    res.check()
    # raster order on the device is asynchronous (the default for device frames); its status words
    # arrive on the stream
    ras = fd.detect_points("shi_tomasi", dev, 200, 20, 40.0)
    assert (ras.frame_flags() & fd.points.FRAME_TIES).all()
    for b in range(2):
        np.testing.assert_array_equal(ras.features(b), oracle.detect(1, host[b], 20, 40.0, 200, sort_mode=1)[0])


def test_reference_order_under_graph_capture(fd, oracle):
    """ties="reference" runs on the GPU (k_select_reference, no host round trip): it captures into a
    hipGraph once its workspace exists, and every replay gives the oracle's std::sort order."""
    torch = pytest.importorskip("torch")
    host = np.stack([make_tie_frame(oracle, seed=s) for s in (11, 12)])
    dev = torch.from_numpy(host).cuda()
    xy = torch.empty((2, 201, 2), dtype=torch.float32, device="cuda")
    cnt = torch.empty((2,), dtype=torch.int32, device="cuda")
    fd.detect_points("harris", dev, 200, 20, 30.0, out=(xy, cnt), ties="reference")  # sizes the workspace
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fd.detect_points("harris", dev, 200, 20, 30.0, out=(xy, cnt), ties="reference")
    for rep in range(3):
        xy.zero_()
        g.replay()
        torch.cuda.synchronize()
        for b in range(2):
            exp = oracle.detect(0, host[b], 20, 30.0, 200, sort_mode=0)[0]
            np.testing.assert_array_equal(xy[b, :int(cnt[b])].cpu().numpy(), exp)


@pytest.mark.parametrize("name", ["harris", "shi_tomasi"])
def test_tie_frames_1080p_batch(fd, oracle, name):
    """The north-star frame size in the reference order: a batch of 1080p tie frames (list-mode
    selection, ~100k+ candidates per frame partitioned on the GPU) next to plain noise frames."""
    frames = np.stack([make_tie_frame(oracle, 1080, 1920, seed=40 + i, copies=(9, 14)) if i % 2 == 0 else
                       oracle.make_frame("noise", 40 + i, 1080, 1920) for i in range(4)])
    _both(fd, oracle, name, frames, 200, 20)
