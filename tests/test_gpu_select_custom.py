"""fd_points_select (SelectGoodFeatures over caller-supplied candidates, the ComputeCandidates seam of
feature_point_detector.h:44) against the oracle's SelectGoodFeatures restatement (oracle.select).

Bar: bit-exact features in both tie orders -- "reference" (libstdc++ std::sort of the pushed sequence,
oracle sort_mode 0) and "raster" (equal responses by raster index, oracle sort_mode 1) -- on lists with
heavy ties (integer gradient magnitudes), in raster / reverse / duplicated push orders, with and
without prior features, for distances 0, 1, 20 and -1."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}
PRIOR = np.array([(i * 15, j * 15) for i in range(1, 10) for j in range(1, 10)], np.float32)


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def gradient_candidates(img, thr=40.0, order="raster"):
    """The C++ demo's custom detector (tests/cpp/test_custom_detector.cpp): |dI/dx| + |dI/dy| > thr."""
    I = img.astype(np.int32)
    gx = np.abs(I[1:-1, 2:] - I[1:-1, :-2])
    gy = np.abs(I[2:, 1:-1] - I[:-2, 1:-1])
    v = (gx + gy).astype(np.float32)
    yy, xx = np.nonzero(v > thr)
    r, x, y = v[yy, xx], (xx + 1).astype(np.int32), (yy + 1).astype(np.int32)
    if order == "reverse":
        r, x, y = r[::-1], x[::-1], y[::-1]
    elif order == "twice":
        r, x, y = np.repeat(r, 2), np.repeat(x, 2), np.repeat(y, 2)
    return np.ascontiguousarray(r), np.ascontiguousarray(x), np.ascontiguousarray(y)


@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_builtin_candidates_through_select(fd, oracle, image_png, name):
    """fd_points_candidates -> fd_points_select gives fd_points_detect's features (both tie orders)."""
    cands = fd.point_candidates(name, image_png, 20, THR[name])
    rows, cols = image_png.shape
    for ties, sm in (("reference", 0), ("raster", 1)):
        res = fd.select_points(cands, rows, cols, 200, 20, ties=ties)
        exp, _ = oracle.detect({"harris": 0, "shi_tomasi": 1, "fast": 2}[name], image_png, 20, THR[name], 200,
                               sort_mode=sm)
        assert np.array_equal(res.features(0), exp), ties


@pytest.mark.parametrize("order", ["raster", "reverse", "twice"])
@pytest.mark.parametrize("dist", [0, 1, 20, -1])
def test_custom_lists_with_ties(fd, oracle, image_png, order, dist):
    rows, cols = image_png.shape
    r, x, y = gradient_candidates(image_png, order=order)
    assert len(r) > 1000
    for prior in (None, PRIOR):
        pr = None if prior is None else [prior]
        for ties, sm in (("reference", 0), ("raster", 1)):
            need = 300 if dist >= 0 else 40
            res = fd.select_points([(r, x, y)], rows, cols, need, dist, prior=pr, ties=ties)
            exp = oracle.select(r, x, y, rows, cols, dist, need, prior, sort_mode=sm)
            assert np.array_equal(res.features(0), exp), (ties, prior is None)
            if ties == "reference":  # device lists: the GPU emulation alone (no host fallback behind it)
                dres = fd.select_points(_dev_lists([(r, x, y)]), rows, cols, need, dist, prior=pr, ties=ties)
                assert np.array_equal(dres.check().features(0), exp), ("device", prior is None)


def _dev_lists(lists):
    import torch

    cap = max(max(len(l[0]) for l in lists), 1)
    t = [torch.zeros((len(lists), cap), dtype=dt) for dt in (torch.float32, torch.int32, torch.int32)]
    for i, l in enumerate(lists):
        for k in range(3):
            t[k][i, :len(l[k])] = torch.from_numpy(np.ascontiguousarray(l[k]))
    counts = torch.tensor([len(l[0]) for l in lists], dtype=torch.int64)
    return tuple(x.cuda() for x in (*t, counts))


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_reference_order_emulation_stress(fd, oracle, seed, wide, monkeypatch):
    """libstdc++'s introsort emulated on the GPU (k_select_reference) on lists with heavy ties: sizes
    around the 16-element threshold and up to 60k, responses from small integer sets (most comparisons
    meet equal keys) or continuous, needs that stop in the first window or run through several (dist 0:
    every visited candidate is kept), with and without the occupancy grid. Device lists, so the GPU
    result stands alone; against the oracle's std::sort (sort_mode 0). wide: the multi-workgroup
    prelude forced on (FD_REF_WIDE=1; by default it runs for frames of >= 1 Mpx only): the 60k list
    goes through three prelude levels before k_select_reference."""
    monkeypatch.setenv("FD_DEBUG_AB", "1")  # (the library reads A/B switches only with it)
    monkeypatch.setenv("FD_REF_WIDE", "1" if wide else "0")
    rng = np.random.default_rng(seed)
    rows, cols = 480, 640
    sizes = [0, 1, 2, 15, 16, 17, 18, 33, 300, 2047, 2049, 5000, 60000]
    lists, needs = [], []
    for n in sizes:
        k = int(rng.integers(1, 40))
        r = (rng.integers(0, k, n).astype(np.float32) if seed % 2 == 0 else rng.standard_normal(n).astype(np.float32))
        idx = rng.permutation(rows * cols)[:n]
        lists.append((r, (idx % cols).astype(np.int32), (idx // cols).astype(np.int32)))
    for dist, need in ((0, 5000), (0, 37), (3, 700), (20, 200)):
        res = fd.select_points(_dev_lists(lists), rows, cols, need, dist, ties="reference")
        res.check()
        for b, (r, x, y) in enumerate(lists):
            exp = oracle.select(r, x, y, rows, cols, dist, need, None, sort_mode=0)
            assert np.array_equal(res.features(b), exp), (sizes[b], dist, need)


def test_batch_device_lists(fd, oracle):
    """Three frames of different list lengths (one empty) as device tensors, features on the device."""
    torch = pytest.importorskip("torch")
    frames = [oracle.make_frame(p, s, 200, 300) for p, s in (("noise", 3), ("checker", 4), ("noise", 5))]
    lists = [gradient_candidates(frames[0]), gradient_candidates(frames[1], order="reverse"),
             (np.zeros(0, np.float32), np.zeros(0, np.int32), np.zeros(0, np.int32))]
    cap = max(len(l[0]) for l in lists) + 5
    resp = torch.zeros((3, cap), dtype=torch.float32)
    xs = torch.zeros((3, cap), dtype=torch.int32)
    ys = torch.zeros((3, cap), dtype=torch.int32)
    for i, (r, x, y) in enumerate(lists):
        resp[i, :len(r)], xs[i, :len(r)], ys[i, :len(r)] = torch.from_numpy(r), torch.from_numpy(x), torch.from_numpy(y)
    counts = torch.tensor([len(l[0]) for l in lists], dtype=torch.int64)
    dev = tuple(t.cuda() for t in (resp, xs, ys, counts))
    res = fd.select_points(dev, 200, 300, 150, 7)  # ties="raster" for device lists
    torch.cuda.synchronize()
    for b, (r, x, y) in enumerate(lists):
        exp = oracle.select(r, x, y, 200, 300, 7, 150, sort_mode=1)
        assert np.array_equal(res.features(b), exp)
    host = fd.select_points(lists, 200, 300, 150, 7)  # host lists: reference order
    for b, (r, x, y) in enumerate(lists):
        assert np.array_equal(host.features(b), oracle.select(r, x, y, 200, 300, 7, 150, sort_mode=0))


def test_full_float_range(fd, oracle):
    """Responses anywhere in the float range (negative, zero, +-inf, denormals) keep their order."""
    rng = np.random.default_rng(3)
    n = 5000
    vals = np.concatenate([rng.standard_normal(n - 6).astype(np.float32) * 1e3,
                           np.array([np.inf, -np.inf, 0.0, -0.0, 1e-42, -1e-42], np.float32)])
    x = rng.integers(0, 640, n).astype(np.int32)
    y = rng.integers(0, 480, n).astype(np.int32)
    for ties, sm in (("reference", 0), ("raster", 1)):
        res = fd.select_points([(vals, x, y)], 480, 640, 400, 3, ties=ties)
        assert np.array_equal(res.features(0), oracle.select(vals, x, y, 480, 640, 3, 400, sort_mode=sm))


def test_invalid_candidates_refused(fd):
    import feature_detector_amd._lib as L

    r = np.array([5.0, 4.0], np.float32)
    for x, y in (((0, 640), (0, 0)), ((0, 1), (-1, 0)), ((0, 1), (0, 480))):
        with pytest.raises(L.FdError):
            fd.select_points([(r, np.array(x, np.int32), np.array(y, np.int32))], 480, 640, 10, 3)
    with pytest.raises(L.FdError):
        fd.select_points([(np.array([1.0, np.nan], np.float32), np.array([1, 2], np.int32),
                           np.array([1, 2], np.int32))], 480, 640, 10, 3)
    # the context keeps working after a refused call
    res = fd.select_points([(r, np.array([1, 9], np.int32), np.array([1, 1], np.int32))], 480, 640, 10, 3)
    assert np.array_equal(res.features(0), np.array([[1, 1], [9, 1]], np.float32))


@pytest.mark.parametrize("n", [40, 200, 1000, 5000, 20000])
def test_reference_order_depth_limit(fd, oracle, n):
    """Candidate lists on which std::sort's introsort reaches its depth limit inside the visited prefix
    (McIlroy's adversary, oracle.introsort_killer: every pivot an extreme, a run of equal responses left
    in the long front range), so the reference's order of those ties is std::__partial_sort's
    (heapsort). k_select flags the frame, k_select_reference emulates the heapsort on the GPU
    (ref_heapsort: in the workgroup levels for the long ranges, in a wave's LDS for <= 256 / <= 64
    elements): device lists, host lists and a graph replay all equal oracle.select(sort_mode=0) -- the
    real std::sort -- and no frame is left unresolved."""
    torch = pytest.importorskip("torch")
    rows, cols = 480, 640
    rng = np.random.default_rng(n)
    r = oracle.introsort_killer(n, True)
    idx = rng.permutation(rows * cols)[:n]
    lst = (r, (idx % cols).astype(np.int32), (idx // cols).astype(np.int32))
    for dist, need in ((3, 200), (0, n), (40, 60)):
        exp = oracle.select(*lst, rows, cols, dist, need, None, sort_mode=0)
        host = fd.select_points([lst], rows, cols, need, dist, ties="reference")
        assert np.array_equal(host.features(0), exp), ("host", dist, need)
        dev = fd.select_points(_dev_lists([lst]), rows, cols, need, dist, ties="reference")
        st = dev.frame_flags()
        assert st[0] & fd.points.FRAME_TIES and st[0] & fd.points.FRAME_RESOLVED, hex(int(st[0]))
        assert not st[0] & fd.points.FRAME_UNRESOLVED
        assert np.array_equal(dev.check().features(0), exp), ("device", dist, need)
    # graph replay (the emulation is capturable: no host round trip)
    dl = _dev_lists([lst])
    xy = torch.empty((1, 201, 2), dtype=torch.float32, device="cuda")
    cnt = torch.empty((1,), dtype=torch.int32, device="cuda")
    fd.select_points(dl, rows, cols, 200, 3, ties="reference", out=(xy, cnt))  # sizes the workspace
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fd.select_points(dl, rows, cols, 200, 3, ties="reference", out=(xy, cnt))
    exp = oracle.select(*lst, rows, cols, 3, 200, None, sort_mode=0)
    for _ in range(2):
        xy.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(xy[0, :int(cnt[0])].cpu().numpy(), exp)


@pytest.mark.parametrize("guard", [1, 2, 4, 12])
def test_reference_order_guard_failure(fd, oracle, image_png, monkeypatch, guard):
    """k_select_reference's window x level loop cut short (FD_REF_GUARD, a diagnostic bound): the frame
    must come out FRAME_UNRESOLVED -- never FRAME_RESOLVED with an unfinished order -- and its device
    features must be either k_select's raster-order selection (no window scanned yet) or a prefix of the
    reference's result, not a mix of the two orders; host outputs fall back to the host sort and equal
    the reference. A frame the bound does not cut stays resolved and equal to the reference."""
    monkeypatch.setenv("FD_DEBUG_AB", "1")
    monkeypatch.setenv("FD_REF_GUARD", str(guard))
    rows, cols = image_png.shape
    lst = gradient_candidates(image_png)  # integer responses: ties fill the visited prefix
    for dist, need in ((20, 200), (3, 2000)):
        exp0 = oracle.select(*lst, rows, cols, dist, need, None, sort_mode=0)
        exp1 = oracle.select(*lst, rows, cols, dist, need, None, sort_mode=1)
        host = fd.select_points([lst], rows, cols, need, dist, ties="reference")
        assert np.array_equal(host.features(0), exp0), ("host", dist, need)
        dev = fd.select_points(_dev_lists([lst]), rows, cols, need, dist, ties="reference")
        st = int(dev.frame_flags()[0])
        got = dev.features(0)
        assert st & fd.points.FRAME_TIES, hex(st)
        if st & fd.points.FRAME_UNRESOLVED:
            assert not st & fd.points.FRAME_RESOLVED, hex(st)
            assert (np.array_equal(got, exp1) or
                    (len(got) < len(exp0) and np.array_equal(got, exp0[:len(got)]))), ("mixed", dist, need, len(got))
        else:
            assert st & fd.points.FRAME_RESOLVED, hex(st)
            assert np.array_equal(got, exp0), ("resolved", dist, need)
    if guard == 1:  # one iteration cannot finish a frame of thousands of candidates
        assert st & fd.points.FRAME_UNRESOLVED, hex(st)
