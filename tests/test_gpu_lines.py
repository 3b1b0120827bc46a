"""GPU: fd_lsd_lines (GPU compact level-line lists + host region growing on worker threads) against
the line oracle (oracle/fd_oracle_lines.cpp). The float sequence is the reference's on both sides, so
the segments are compared bit for bit (all 12 rectangle fields), not just within SURVEY §8c's 0.5 px."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(fd, oracle, frames, threads=0):
    frames = np.ascontiguousarray(frames)
    got = fd.lsd_lines(frames, threads=threads)
    for b in range(frames.shape[0]):
        exp = oracle.lsd_lines(frames[b])
        assert got[b].shape == exp.shape, (b, got[b].shape, exp.shape)
        assert np.array_equal(got[b].view(np.uint32), exp.view(np.uint32)), b
    return got


def test_image_png(image_png, oracle):
    import feature_detector_amd as fd

    got = _check(fd, oracle, image_png[None])
    assert len(got[0]) == 40


@pytest.mark.parametrize("rows,cols,expect", [(480, 640, 112), (1080, 1920, 792)])
def test_checker64(oracle, rows, cols, expect):
    import feature_detector_amd as fd

    img = oracle.make_frame("checker", 1234, rows, cols, 64)
    assert len(_check(fd, oracle, img[None])[0]) == expect


def test_batch_threads_and_patterns(oracle):
    import feature_detector_amd as fd

    frames = np.stack([oracle.make_frame(p, s, 240, 320, per) for p, s, per in
                       (("checker", 1, 16), ("noise", 2, 16), ("checker", 3, 40), ("checker", 4, 64),
                        ("noise", 5, 16), ("checker", 6, 24))])
    one = _check(fd, oracle, frames, threads=1)
    many = fd.lsd_lines(frames, threads=4)
    assert all(np.array_equal(a, b) for a, b in zip(one, many))


def test_ragged_and_tiny(oracle):
    import feature_detector_amd as fd

    rng = np.random.default_rng(7)
    for shape in ((37, 53), (61, 200), (5, 5), (4, 4), (3, 3), (2, 2), (2, 9), (9, 2)):
        img = (rng.integers(0, 4, shape) * 60).astype(np.uint8)
        _check(fd, oracle, img[None])


def test_ring_overflow_ramp(oracle):
    import feature_detector_amd as fd

    r, c = np.mgrid[0:400, 0:600]
    img = ((r * 3 + c * 5) % 256).astype(np.uint8)
    _check(fd, oracle, img[None])


def test_needed_zero(image_png):
    import feature_detector_amd as fd

    assert len(fd.lsd_lines(image_png[None], needed=0)[0]) == 0


def test_device_input_matches_host(oracle):
    import torch

    import feature_detector_amd as fd

    img = oracle.make_frame("checker", 9, 480, 640, 32)
    host = fd.lsd_lines(img[None])
    dev = fd.lsd_lines(torch.from_numpy(img[None]).cuda())
    assert np.array_equal(host[0], dev[0])


def test_config4_batch_spot_check(oracle):
    # BASELINE configs[3] shape: 256 frames of 1920x1080; frames 0, 127 and 255 against the oracle,
    # every frame's segments within the frame and of length >= 20
    import torch

    import feature_detector_amd as fd

    g = torch.Generator(device="cuda")
    g.manual_seed(4242)
    rows, cols, n = 1080, 1920, 256
    r = torch.arange(rows, device="cuda").view(1, rows, 1) // 64
    c = torch.arange(cols, device="cuda").view(1, 1, cols) // 64
    base = torch.where(((r + c) % 2) == 1, 180, 60)
    noise = torch.randint(-10, 11, (n, rows, cols), generator=g, device="cuda", dtype=torch.int32)
    frames = (base + noise).clamp(0, 255).to(torch.uint8)
    got = fd.lsd_lines(frames, max_lines=8192)
    assert len(got) == n
    host = frames.cpu().numpy()
    for b in (0, 127, 255):
        exp = oracle.lsd_lines(host[b])
        assert np.array_equal(got[b].view(np.uint32), exp.view(np.uint32)), b
    for seg in got:
        assert len(seg) > 0 and (seg[:, 6] >= 20).all()
        assert (seg[:, [0, 2]] > -2).all() and (seg[:, [0, 2]] < cols + 2).all()


def test_seed_order_on_gpu(oracle, monkeypatch, capfd):
    # the seed order (sorted_pixels_, feature_line_detector.cpp:88-94) comes from the GPU
    # (k_select_reference in push order) for every frame, including a ramp whose norms are all equal
    # (the introsort's equal-key paths) and a 1080p frame; the segments are the oracle's and those of
    # the host std::sort (FD_LSD_HOST_SORT=1), and with the multi-workgroup prelude (FD_LSD_WIDE=1) or
    # the order through a device buffer (FD_LSD_ORD_MAPPED=0) the same
    import feature_detector_amd as fd

    r, c = np.mgrid[0:400, 0:600]
    ramp = ((r * 3 + c * 5) % 256).astype(np.uint8)
    small = np.stack([ramp, oracle.make_frame("checker", 11, 400, 600, 24), oracle.make_frame("noise", 12, 400, 600, 16)])
    big = oracle.make_frame("checker", 13, 1080, 1920, 64)[None]
    monkeypatch.setenv("FD_DEBUG_AB", "1")
    monkeypatch.setenv("FD_LINES_TIMING", "1")
    for frames in (small, big):
        capfd.readouterr()
        got = _check(fd, oracle, frames)
        err = capfd.readouterr().err
        assert f"seed orders from the gpu {frames.shape[0]}" in err, err
        monkeypatch.setenv("FD_LSD_HOST_SORT", "1")
        host = fd.lsd_lines(frames)
        assert "seed orders from the gpu 0" in capfd.readouterr().err
        monkeypatch.delenv("FD_LSD_HOST_SORT")
        assert all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(got, host))
        # the order through a device buffer and a copy instead of written into pinned host memory
        monkeypatch.setenv("FD_LSD_ORD_MAPPED", "0")
        copied = fd.lsd_lines(frames)
        assert f"seed orders from the gpu {frames.shape[0]}" in capfd.readouterr().err
        monkeypatch.delenv("FD_LSD_ORD_MAPPED")
        assert all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(got, copied))
        monkeypatch.setenv("FD_LSD_WIDE", "1")
        wide = fd.lsd_lines(frames)
        assert f"seed orders from the gpu {frames.shape[0]}" in capfd.readouterr().err
        monkeypatch.delenv("FD_LSD_WIDE")
        assert all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(got, wide))


def test_seed_order_guard_failure_falls_back(oracle, monkeypatch, capfd):
    # the seed sort's loop bound cut short (FD_REF_GUARD, diagnostic) right after a full GPU call of the
    # same frames: every frame must be reported unresolved -- not resolved with the previous call's order
    # still in the pinned buffer's tail -- and be sorted on the host, with the oracle's segments
    import feature_detector_amd as fd

    frames = np.stack([oracle.make_frame("checker", 21, 400, 600, 24), oracle.make_frame("noise", 22, 400, 600, 16)])
    monkeypatch.setenv("FD_DEBUG_AB", "1")
    monkeypatch.setenv("FD_LINES_TIMING", "1")
    capfd.readouterr()
    full = _check(fd, oracle, frames)
    assert f"seed orders from the gpu {frames.shape[0]}" in capfd.readouterr().err
    for guard in (1, 3):
        monkeypatch.setenv("FD_REF_GUARD", str(guard))
        got = _check(fd, oracle, frames)
        assert "seed orders from the gpu 0" in capfd.readouterr().err
        assert all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(got, full))
