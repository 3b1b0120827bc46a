"""GPU parity of the steered-BRIEF kernel (fd_brief_compute) against the CPU oracle.

Bar: bit-exact descriptor words and valid flags against oracle.brief for both sampler restatements
(the reference's float sampler is un-vendored, so the sampled bits are "parity unpinned"; the border
test, moments, orientation and rotated coordinates are the reference's exact float sequence).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def oracle_batch(oracle, frames, uv, counts, length, half, sampler):
    B, S = uv.shape[:2]
    nw = (length + 31) // 32
    bits = np.zeros((B, S, nw), np.uint32)
    valid = np.zeros((B, S), np.uint8)
    for b in range(B):
        n = S if counts is None else int(counts[b])
        if n:
            bb, vv, _ = oracle.brief(frames[b], uv[b, :n], length, half, sampler)
            bits[b, :n], valid[b, :n] = bb, vv
    return bits, valid


@pytest.mark.parametrize("sampler", ["bilinear", "truncate"])
def test_demo_config_image_png(fd, oracle, image_png, sampler):
    """test_feature_descriptor.cpp:16-57: Harris thr 20, dist 20, need 10, then BRIEF kLength 128, half 8."""
    res = fd.detect_points("harris", image_png, 10, 20, 20.0)
    xy = res.features(0)
    assert len(xy) == 10
    bits, valid = fd.brief_compute(image_png, xy, length=128, half_patch_size=8, sampler=sampler, with_valid=True)
    eb, ev, _ = oracle.brief(image_png, xy, 128, 8, 0 if sampler == "bilinear" else 1)
    assert np.array_equal(valid[0], ev)
    assert np.array_equal(bits[0], eb)


@pytest.mark.parametrize("sampler", [0, 1])
@pytest.mark.parametrize("length,half", [(256, 8), (1, 8), (31, 4), (32, 0), (33, 1), (100, 15), (255, 31),
                                         (256, 32), (64, 40)])
def test_fractional_keypoints(fd, oracle, sampler, length, half):
    rng = np.random.default_rng(length * 131 + half)
    frames = np.stack([oracle.make_frame("noise", 50 + i, 240, 280) for i in range(2)])
    S = 24
    uv = np.stack([rng.uniform(-5, 290, (S, 2)) for _ in range(2)]).astype(np.float32)
    uv[..., 1] *= 240.0 / 280.0
    uv[:, :6] = np.round(uv[:, :6])  # integral keypoints take the exact-integer moment path
    uv[0, 6] = (np.nan, 50.0)
    uv[1, 7] = (100.0, np.inf)
    bits, valid = fd.brief_compute(frames, uv, length=length, half_patch_size=half, sampler=sampler, with_valid=True)
    eb, ev = oracle_batch(oracle, frames, uv, None, length, half, sampler)
    assert np.array_equal(valid, ev)
    assert np.array_equal(bits, eb)
    # half 0: the patch is the keypoint alone, m10 = m01 = 0, so every descriptor is zero (:30)
    assert (valid.sum() > 0) if half > 0 else (valid.sum() == 0)


def test_counts_and_unwritten_slots(fd, oracle):
    frames = np.stack([oracle.make_frame("checker", 9 + i, 120, 160) for i in range(3)])
    rng = np.random.default_rng(3)
    uv = rng.uniform(20, 100, (3, 10, 2)).astype(np.float32)
    counts = np.array([10, 0, 4], np.int32)
    L = fd.load()
    import ctypes
    from feature_detector_amd._lib import fd_brief_opts

    ctx = fd.default_context()
    ctx.set_stream(None)
    bits = np.full((3, 10, 8), 0xDEADBEEF, np.uint32)
    valid = np.full((3, 10), 7, np.uint8)
    opts = fd_brief_opts(256, 8, 0)
    rc = L.fd_brief_compute(ctx.ptr, ctypes.c_void_p(frames.ctypes.data), 0, 3, 120, 160, ctypes.byref(opts),
                            ctypes.c_void_p(uv.ctypes.data), ctypes.c_void_p(counts.ctypes.data), 10,
                            ctypes.c_void_p(bits.ctypes.data), ctypes.c_void_p(valid.ctypes.data), 0)
    assert rc == 0
    eb, ev = oracle_batch(oracle, frames, uv, counts, 256, 8, 0)
    for b in range(3):
        n = counts[b]
        assert np.array_equal(bits[b, :n], eb[b, :n]) and np.array_equal(valid[b, :n], ev[b, :n])
        assert (bits[b, n:] == 0xDEADBEEF).all() and (valid[b, n:] == 7).all()


def test_bad_arguments(fd, oracle):
    img = oracle.make_frame("noise", 1, 64, 64)
    uv = np.array([[32, 32]], np.float32)
    for kw in ({"length": 0}, {"length": 257}, {"half_patch_size": -1}, {"sampler": 5}):
        with pytest.raises(fd.FdError):
            fd.brief_compute(img, uv, **kw)


def test_device_chain_fast_720p(fd, oracle):
    """Config 3 shape (FAST + BRIEF-256, 1280x720) on a small batch: detect writes device keypoints,
    BRIEF reads them (and detect's device counts) in place, no host round trip in between."""
    torch = pytest.importorskip("torch")
    B = 4
    host = np.stack([oracle.make_frame("checker" if i % 2 else "noise", 700 + i, 720, 1280) for i in range(B)])
    dev = torch.from_numpy(host).cuda()
    res = fd.detect_points("fast", dev, 500, 15, 10.0)
    bits, valid = fd.brief_compute(dev, res.xy, res.counts, length=256, half_patch_size=8, with_valid=True)
    torch.cuda.synchronize()
    counts = res.counts.cpu().numpy()
    xy = res.xy.cpu().numpy()
    bits = bits.cpu().numpy().view(np.uint32)
    valid = valid.cpu().numpy()
    assert counts.min() > 0
    for b in range(B):
        n = counts[b]
        eb, ev, _ = oracle.brief(host[b], xy[b, :n], 256, 8, 0)
        assert np.array_equal(valid[b, :n], ev)
        assert np.array_equal(bits[b, :n], eb)


def test_descriptor_helpers(fd, oracle):
    img = oracle.make_frame("noise", 4, 100, 100)
    uv = np.array([[50, 50], [5, 5]], np.float32)
    bits = fd.brief_compute(img, uv, length=40)
    b = fd.unpack_bits(bits[0], 40)
    f = fd.to_float(bits[0], 40)
    assert b.shape == (2, 40) and f.shape == (2, 40)
    assert np.array_equal(f[0], np.where(b[0], 1.0, -1.0))
    assert not b[1].any() and (f[1] == -1.0).all()  # out of border: all-zero bits -> all -1.0f
