"""GPU parity of the point-detection hot path (HIP kernels via the C ABI) against the CPU oracle.

Bar: bit-exact. Candidates (response bits, x, y, raster order) and the Harris/Shi-Tomasi response
maps must equal the oracle's; selected features must equal the oracle's in both tie orders: the
default "reference" order (the reference's std::sort permutation) against oracle sort_mode 0, and
"raster" (response desc, raster asc) against the oracle's stable order (sort_mode 1).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2}
THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def build_mask(rows, cols, dist, prior):
    """feature_point_detector.cpp:12-16, :76-98 (boxes around truncated prior features)."""
    m = np.ones((rows, cols), np.int32)
    for x, y in np.asarray(prior, np.float32).reshape(-1, 2):
        r0, c0 = int(np.float32(y)), int(np.float32(x))
        m[max(r0 - dist, 0):max(min(r0 + dist, rows - 1) + 1, 0), max(c0 - dist, 0):max(min(c0 + dist, cols - 1) + 1, 0)] = 0
    return m


def oracle_candidates(oracle, name, img, thr, mask=None):
    if name == "fast":
        return oracle.fast_candidates(img, thr, mask)
    resp = oracle.response_map(img, KIND[name], thr, mask)
    return oracle.nms(resp, thr)


def assert_same_candidates(got, exp):
    gr, gx, gy = got
    er, ex, ey = exp
    assert len(gr) == len(er)
    assert np.array_equal(gx, ex) and np.array_equal(gy, ey)
    assert np.array_equal(gr.view(np.uint32), er.view(np.uint32))


def check_detect(fd, oracle, name, img, dist, thr, need, prior=None):
    pr = None if prior is None else [prior]
    res = fd.detect_points(name, img, need, dist, thr, prior=pr)  # ties="reference"
    got = res.features(0)
    exp_ref, cands_ref = oracle.detect(KIND[name], img, dist, thr, need, prior, sort_mode=0)
    assert np.array_equal(got, exp_ref)
    raster = fd.detect_points(name, img, need, dist, thr, prior=pr, ties="raster")
    exp_stable, _ = oracle.detect(KIND[name], img, dist, thr, need, prior, sort_mode=1)
    assert np.array_equal(raster.features(0), exp_stable)
    if not np.array_equal(exp_ref, exp_stable):
        # Only possible when equal responses meet inside the scanned prefix (unstable std::sort),
        # and then the GPU must have flagged the frame and re-selected it in the reference order.
        assert oracle.prefix_has_ties(cands_ref[0], len(cands_ref[0]))
        assert res.frame_flags()[0] & fd.points.FRAME_RESOLVED
    return got


# ------------------------------------------------------------------ reference demo image (golden)

@pytest.mark.parametrize("name", ["fast", "harris", "shi_tomasi"])
def test_image_png_candidates_bit_exact(fd, oracle, image_png, ref_counts, name):
    thr = THR[name]
    (got,), rmap = fd.point_candidates(name, image_png, 20, thr, response_map=True)
    exp = oracle_candidates(oracle, name, image_png, thr)
    assert_same_candidates(got, exp)
    assert len(got[0]) == ref_counts["image_png"][name]["candidates"]
    if name != "fast":
        eresp = oracle.response_map(image_png, KIND[name], thr)
        assert np.array_equal(rmap[0].view(np.uint32), eresp.view(np.uint32))


@pytest.mark.parametrize("name", ["fast", "harris", "shi_tomasi"])
def test_image_png_features(fd, oracle, image_png, ref_counts, name):
    got = check_detect(fd, oracle, name, image_png, 20, THR[name], 200)
    assert len(got) == ref_counts["image_png"][name]["features"]


def test_image_png_prior_lattice(fd, oracle, image_png):
    # TestUpdateMaskWithDetectedFeatures (test/test_feature_point_detector.cpp:44-65): 81 priors.
    prior = np.array([(i * 15, j * 15) for i in range(1, 10) for j in range(1, 10)], np.float32)
    for name in ("harris", "shi_tomasi", "fast"):
        check_detect(fd, oracle, name, image_png, 20, THR[name], 200, prior)
        (got,) = fd.point_candidates(name, image_png, 20, THR[name], prior=[prior])
        exp = oracle_candidates(oracle, name, image_png, THR[name], build_mask(480, 752, 20, prior))
        assert_same_candidates(got, exp)


# ------------------------------------------------------------------ seeded synthetic frames

@pytest.mark.parametrize("size", [(480, 640), (720, 1280)])
@pytest.mark.parametrize("pattern", ["noise", "checker"])
@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_synthetic_bit_exact(fd, oracle, ref_counts, size, pattern, name):
    rows, cols = size
    img = oracle.make_frame(pattern, 1234, rows, cols)
    (got,), rmap = fd.point_candidates(name, img, 20, THR[name], response_map=True)
    exp = oracle_candidates(oracle, name, img, THR[name])
    assert_same_candidates(got, exp)
    rec = [r for r in ref_counts["synthetic_candidates"]
           if r["rows"] == rows and r["cols"] == cols and r["pattern"] == pattern][0]
    assert len(got[0]) == rec[name]
    if name != "fast":
        eresp = oracle.response_map(img, KIND[name], THR[name])
        assert np.array_equal(rmap[0].view(np.uint32), eresp.view(np.uint32))
    check_detect(fd, oracle, name, img, 20, THR[name], 200)


def test_batch_equals_single(fd, oracle):
    frames = np.stack([oracle.make_frame(p, s, 240, 320) for p, s in
                       (("noise", 1), ("checker", 2), ("noise", 3), ("checker", 4))])
    for name in ("harris", "shi_tomasi", "fast"):
        res = fd.detect_points(name, frames, 100, 10, THR[name])
        for b in range(len(frames)):
            single = fd.detect_points(name, frames[b], 100, 10, THR[name]).features(0)
            assert np.array_equal(res.features(b), single)
            exp, _ = oracle.detect(KIND[name], frames[b], 10, THR[name], 100, sort_mode=0)
            assert np.array_equal(single, exp)


# ------------------------------------------------------------------ edge cases

@pytest.mark.parametrize("shape", [(1, 1), (4, 4), (5, 5), (6, 7), (7, 7), (8, 9), (13, 250), (250, 13),
                                   (33, 257), (479, 641), (61, 253)])
@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_ragged_shapes(fd, oracle, shape, name):
    rows, cols = shape
    img = oracle.make_frame("noise", 7 + rows * cols, rows, cols)
    thr = THR[name]
    (got,) = fd.point_candidates(name, img, 3, thr)
    assert_same_candidates(got, oracle_candidates(oracle, name, img, thr))
    check_detect(fd, oracle, name, img, 3, thr, 50)


@pytest.mark.parametrize("dist,need", [(0, 200), (1, 300), (2, 64), (20, 0), (20, 1), (100, 1000), (-1, 30)])
@pytest.mark.parametrize("name", ["harris", "fast"])
def test_distance_and_need_edges(fd, oracle, name, dist, need):
    img = oracle.make_frame("noise", 99, 480, 640)
    check_detect(fd, oracle, name, img, dist, THR[name], need)


@pytest.mark.parametrize("thr", [-1.0, 0.0, 0.1, 1e6])
@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_thresholds(fd, oracle, name, thr):
    img = oracle.make_frame("checker", 5, 120, 160)
    (got,) = fd.point_candidates(name, img, 15, thr)
    assert_same_candidates(got, oracle_candidates(oracle, name, img, thr))
    check_detect(fd, oracle, name, img, 15, thr, 40)


def test_priors_exceeding_need(fd, oracle, image_png):
    # features.size() >= need is checked only after an append (feature_point_detector.cpp:67-69):
    # with 81 priors and need 10, exactly one new feature is added.
    prior = np.array([(i * 15, j * 15) for i in range(1, 10) for j in range(1, 10)], np.float32)
    got = check_detect(fd, oracle, "harris", image_png, 20, 30.0, 10, prior)
    assert len(got) == 1


def test_priors_out_of_image_and_fractional(fd, oracle):
    img = oracle.make_frame("noise", 11, 200, 300)
    prior = np.array([(-5.7, 3.2), (299.9, 199.9), (150.5, 100.5), (1000, 1000), (0.0, 0.0)], np.float32)
    for name in ("harris", "fast"):
        check_detect(fd, oracle, name, img, 12, THR[name], 80, prior)


def test_empty_candidates(fd, oracle):
    img = np.full((64, 64), 128, np.uint8)
    for name in ("harris", "shi_tomasi", "fast"):
        res = fd.detect_points(name, img, 200, 20, THR[name])
        assert int(res.counts[0]) == 0


# ------------------------------------------------------------------ full size (north-star shape)

@pytest.mark.parametrize("name", ["shi_tomasi", "harris", "fast"])
def test_1080p_against_oracle_and_golden_counts(fd, oracle, ref_counts, name):
    frames = np.stack([oracle.make_frame(p, 1234, 1080, 1920) for p in ("noise", "checker")])
    res = fd.detect_points(name, frames, 200, 20, THR[name])
    for b, p in enumerate(("noise", "checker")):
        exp, cands = oracle.detect(KIND[name], frames[b], 20, THR[name], 200, sort_mode=0)
        rec = [r for r in ref_counts["synthetic_candidates"]
               if r["rows"] == 1080 and r["pattern"] == p][0]
        assert len(cands[0]) == rec[name]
        assert np.array_equal(res.features(b), exp)


def test_large_batch_properties(fd, oracle):
    """Size-independent invariants on a 64-frame 1080p batch: per-frame determinism under batching,
    greedy invariants (pairwise Chebyshev distance > d, count == need), and spot parity."""
    torch = pytest.importorskip("torch")
    B = 64
    host = np.stack([oracle.make_frame("noise" if i % 2 == 0 else "checker", 1000 + i, 1080, 1920)
                     for i in range(B)])
    dev = torch.from_numpy(host).cuda()
    res = fd.detect_points("shi_tomasi", dev, 200, 20, 40.0, ties="reference")
    torch.cuda.synchronize()
    counts = res.counts.cpu().numpy()
    xy = res.xy.cpu().numpy()
    assert (counts == 200).all()
    for b in range(B):
        f = xy[b, :counts[b]]
        d = np.abs(f[:, None, :] - f[None, :, :]).max(-1)
        np.fill_diagonal(d, 1e9)
        assert d.min() > 20
    for b in (0, 1, 37):
        exp, _ = oracle.detect(1, host[b], 20, 40.0, 200, sort_mode=0)
        assert np.array_equal(xy[b, :counts[b]], exp)


def test_device_tensor_path_matches_host(fd, oracle):
    torch = pytest.importorskip("torch")
    frames = np.stack([oracle.make_frame("noise", s, 480, 640) for s in (21, 22, 23)])
    for name in ("harris", "shi_tomasi", "fast"):
        hres = fd.detect_points(name, frames, 200, 20, THR[name])
        dres = fd.detect_points(name, torch.from_numpy(frames).cuda(), 200, 20, THR[name], ties="reference")
        torch.cuda.synchronize()
        assert np.array_equal(dres.counts.cpu().numpy(), hres.counts)
        for b in range(3):
            assert np.array_equal(dres.features(b), hres.features(b))


@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_point_response_and_append(fd, oracle, name):
    """fd_points_response (unordered candidates) equals the oracle's candidate set; the append
    variant (no count reset) adds a second copy after the first."""
    torch = pytest.importorskip("torch")
    frames = np.stack([oracle.make_frame(p, s, 240, 320) for p, s in (("noise", 5), ("checker", 6))])
    dev = torch.from_numpy(frames).cuda()
    resp, idx, cnt = fd.point_response(name, dev, THR[name])
    torch.cuda.synchronize()
    cnt = cnt.cpu().numpy()
    cap = resp.shape[1]
    for b in range(2):
        er, ex, ey = oracle_candidates(oracle, name, frames[b], THR[name])
        gi = idx[b, :cnt[b]].cpu().numpy()
        gr = resp[b, :cnt[b]].cpu().numpy()
        order = np.argsort(gi, kind="stable")
        assert np.array_equal(gi[order], ey.astype(np.int64) * 320 + ex)
        assert np.array_equal(gr[order].view(np.uint32), er.view(np.uint32))
    big = (torch.empty((2, 2 * cap), dtype=torch.float32, device="cuda"),
           torch.empty((2, 2 * cap), dtype=torch.int32, device="cuda"),
           torch.zeros((2,), dtype=torch.int32, device="cuda"))
    fd.point_response(name, dev, THR[name], out=big, append=True)
    fd.point_response(name, dev, THR[name], out=big, append=True)
    torch.cuda.synchronize()
    c2 = big[2].cpu().numpy()
    assert np.array_equal(c2, 2 * cnt)
    for b in range(2):
        gi = np.sort(big[1][b, :c2[b]].cpu().numpy())
        assert np.array_equal(gi[0::2], gi[1::2])
    with pytest.raises(ValueError):
        fd.point_response(name, dev, THR[name], append=True)


def test_point_response_huge_capacity(fd, oracle):
    """cand_cap >= 2^30 on a launch large enough for the lane-wide kernel (1024x2048, 2^21 px): the
    library must not address the caller's list through a 32-bit buffer range (2^30 * 4 B wraps to 0);
    the list still equals the oracle's candidate set. 8 GiB of HBM for the two list arrays."""
    torch = pytest.importorskip("torch")
    img = oracle.make_frame("noise", 77, 1024, 2048)
    dev = torch.from_numpy(np.ascontiguousarray(img[None])).cuda()
    cap = 1 << 30
    out = (torch.empty((1, cap), dtype=torch.float32, device="cuda"),
           torch.empty((1, cap), dtype=torch.int32, device="cuda"),
           torch.empty((1,), dtype=torch.int32, device="cuda"))
    resp, idx, cnt = fd.point_response("shi_tomasi", dev, THR["shi_tomasi"], out=out)
    torch.cuda.synchronize()
    n = int(cnt.cpu()[0])
    er, ex, ey = oracle_candidates(oracle, "shi_tomasi", img, THR["shi_tomasi"])
    assert n == len(er)
    gi = idx[0, :n].cpu().numpy().astype(np.int64)
    gr = resp[0, :n].cpu().numpy()
    o = np.argsort(gi, kind="stable")
    assert np.array_equal(gi[o], ey.astype(np.int64) * 2048 + ex)
    assert np.array_equal(gr[o].view(np.uint32), er.view(np.uint32))
    del out, resp, idx
    torch.cuda.empty_cache()


def test_sqrt_rsq_exhaustive():
    # The Shi-Tomasi kernel's sqrt (fd_device.h sqrt_rn_rsq2: v_rsq_f32 + one Newton step) equals the
    # correctly rounded sqrt on every float of its domain ({0} U [2^-60, FLT_MAX], ~1.6e9 values).
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "calib", "sqrt_exhaustive")
    assert os.path.exists(exe), "build tools/calib first (__graft_entry__.build())"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and " 0 mismatches" in out.stdout, out.stdout + out.stderr


@pytest.mark.parametrize("name,size", [("fast", (720, 1280)), ("shi_tomasi", (1080, 1920)), ("harris", (1080, 1920))])
def test_priors_long_scans(fd, oracle, name, size):
    """Prior features on the long-scan paths (FAST, and list-mode frames >= 1 Mpx): the selection's
    grid prefilter is active from the first sub-chunk, with a dense prior lattice, dist 20 and a
    need that forces several sub-chunks; both tie orders against the oracle."""
    rows, cols = size
    img = oracle.make_frame("noise", 4321, rows, cols)
    prior = np.array([(x, y) for x in range(37, cols, 97) for y in range(41, rows, 89)], np.float32)
    check_detect(fd, oracle, name, img, 20, THR[name], len(prior) + 150, prior)


@pytest.mark.parametrize("px", ["0", "2", "4", "8"])
def test_lane_widths_bit_exact(fd, oracle, image_png, monkeypatch, px):
    """Every per-pixel kernel variant (FD_PX: 0 = k_corner, 2/4/8 = k_corner_lp columns per lane; the
    library picks one by launch size) gives the oracle's unordered candidate set and, through detect
    (sorted-segment and list modes, with and without priors), the oracle's features."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("FD_DEBUG_AB", "1")  # (the library reads A/B switches only with it)
    monkeypatch.setenv("FD_PX", px)
    frames = [image_png, oracle.make_frame("noise", 31, 480, 640), oracle.make_frame("checker", 32, 250, 13),
              oracle.make_frame("noise", 33, 37, 1001)]
    for img in frames:
        rows, cols = img.shape
        dev = torch.from_numpy(np.ascontiguousarray(img[None])).cuda()
        for name in ("harris", "shi_tomasi"):
            resp, idx, cnt = fd.point_response(name, dev, THR[name])
            torch.cuda.synchronize()
            n = int(cnt.cpu()[0])
            gi = idx[0, :n].cpu().numpy().astype(np.int64)
            gr = resp[0, :n].cpu().numpy()
            er, ex, ey = oracle_candidates(oracle, name, img, THR[name])
            o = np.argsort(gi, kind="stable")
            assert np.array_equal(gi[o], ey.astype(np.int64) * cols + ex)
            assert np.array_equal(gr[o].view(np.uint32), er.view(np.uint32))
            check_detect(fd, oracle, name, img, 20, THR[name], 200)
    prior = np.array([(x, y) for x in range(20, 752, 60) for y in range(15, 480, 45)], np.float32)
    check_detect(fd, oracle, "shi_tomasi", image_png, 15, 40.0, len(prior) + 120, prior)


def _full_list_check(fd, oracle, name, frames):
    """fd_points_response's whole unordered candidate list of every frame equals the oracle's
    candidate set (sorted by raster index), bit for bit."""
    torch = pytest.importorskip("torch")
    B, rows, cols = frames.shape
    dev = torch.from_numpy(frames).cuda()
    resp, idx, cnt = fd.point_response(name, dev, THR[name])
    torch.cuda.synchronize()
    cnt = cnt.cpu().numpy()
    for b in range(B):
        er, ex, ey = oracle_candidates(oracle, name, frames[b], THR[name])
        assert cnt[b] == len(er), (name, b, cnt[b], len(er))
        gi = idx[b, :cnt[b]].cpu().numpy().astype(np.int64)
        gr = resp[b, :cnt[b]].cpu().numpy()
        o = np.argsort(gi, kind="stable")
        assert np.array_equal(gi[o], ey.astype(np.int64) * cols + ex)
        assert np.array_equal(gr[o].view(np.uint32), er.view(np.uint32))
    return dev


@pytest.mark.parametrize("name", ["shi_tomasi", "harris"])
def test_full_lists_north_star_shape(fd, oracle, name):
    """The timed per-pixel kernel at the north-star frame size (1920x1080, 8 frames of noise and checker:
    a launch large enough for the list-mode kernel and its flushes): full candidate lists against the
    oracle, then every frame's features through detect."""
    frames = np.stack([oracle.make_frame("noise" if i % 2 == 0 else "checker", 900 + i, 1080, 1920) for i in range(8)])
    dev = _full_list_check(fd, oracle, name, frames)
    res = fd.detect_points(name, dev, 200, 20, THR[name], ties="reference")
    for b in range(len(frames)):
        exp, _ = oracle.detect(KIND[name], frames[b], 20, THR[name], 200, sort_mode=0)
        assert np.array_equal(res.features(b), exp)


def test_full_lists_fast_720p(fd, oracle):
    """k_fast at the configs[2] frame size (1280x720, 8 noise frames: ~30 % of the pixels are candidates,
    many staging flushes): full candidate lists against the oracle, and every frame's features."""
    frames = np.stack([oracle.make_frame("noise", 950 + i, 720, 1280) for i in range(8)])
    dev = _full_list_check(fd, oracle, "fast", frames)
    res = fd.detect_points("fast", dev, 200, 20, THR["fast"], ties="reference")
    for b in range(len(frames)):
        exp, _ = oracle.detect(2, frames[b], 20, THR["fast"], 200, sort_mode=0)
        assert np.array_equal(res.features(b), exp)
