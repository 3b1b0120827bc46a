"""GPU parity of the LSD level-line map (fd_lsd_map) against the oracle: bit-exact norm, valid flag
and angle (the kernel restates glibc's fdlibm atan2f), and the column-major valid list in the
reference's scan order (sorted_pixels_ before its std::sort, feature_line_detector.cpp:71-92)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def check_lsd(fd, oracle, img, min_norm=20.0):
    (n, a, v, idx), = fd.lsd_map(img, min_norm)
    en, ea, ev, eidx = oracle.lsd_map(img, min_norm)
    assert np.array_equal(n.view(np.uint32), en.view(np.uint32))
    assert np.array_equal(v, ev)
    assert np.array_equal(a.view(np.uint32), ea.view(np.uint32))
    assert np.array_equal(idx, eidx)
    # host std::sort of the GPU list reproduces the reference's sorted_pixels_ exactly
    assert np.array_equal(oracle.lsd_sort(n, idx, 0), oracle.lsd_sort(en, eidx, 0))
    return idx


def test_image_png(fd, oracle, image_png, ref_counts):
    idx = check_lsd(fd, oracle, image_png)
    assert len(idx) == ref_counts["image_png"]["lsd_valid"]


@pytest.mark.parametrize("rec_i", [0, 1, 2])
def test_synthetic_counts(fd, oracle, ref_counts, rec_i):
    rec = ref_counts["synthetic_lsd_valid"][rec_i]
    img = oracle.make_frame(rec["pattern"], 1234, rec["rows"], rec["cols"], rec["period"])
    idx = check_lsd(fd, oracle, img)
    assert len(idx) == rec["valid"]


@pytest.mark.parametrize("shape", [(2, 2), (3, 3), (4, 4), (5, 67), (67, 5), (100, 129), (257, 63)])
def test_ragged(fd, oracle, shape):
    img = np.random.default_rng(shape[0] * 1000 + shape[1]).integers(0, 256, shape, dtype=np.uint8)
    check_lsd(fd, oracle, img, 20.0)


@pytest.mark.parametrize("min_norm", [0.0, 5.0, 100.0, 400.0])
def test_thresholds(fd, oracle, min_norm):
    img = np.random.default_rng(3).integers(0, 256, (120, 200), dtype=np.uint8)
    check_lsd(fd, oracle, img, min_norm)


def test_angle_domain_exhaustive(fd, oracle):
    """Every (ad, bc) gradient pair -> every half-integer (gx, gy): built as 2x2 blocks."""
    vals = []
    for ad in range(-255, 256):
        for bc in range(-255, 256):
            # I(r,c)=p, I(r+1,c+1)=p+ad, I(r,c+1)=q, I(r+1,c)=q-bc with values in [0,255]
            p = max(0, -ad)
            q = max(0, bc)
            if p + ad > 255 or q - bc > 255 or q > 255:
                continue
            vals.append((p, q, q - bc, p + ad))
    n = len(vals)
    img = np.zeros((3, 2 * n + 2), np.uint8)
    for i, (a, b, c, d) in enumerate(vals):
        img[1, 1 + 2 * i], img[1, 2 + 2 * i] = a, b
        img[2, 1 + 2 * i], img[2, 2 + 2 * i] = c, d
    img = np.concatenate([img, np.zeros((2, img.shape[1]), np.uint8)])
    check_lsd(fd, oracle, img, 0.0)


def test_batch(fd, oracle):
    frames = np.stack([oracle.make_frame("checker", s, 240, 320, 32) for s in range(5)])
    res = fd.lsd_map(frames)
    for b in range(5):
        en, ea, ev, eidx = oracle.lsd_map(frames[b])
        assert np.array_equal(res[b][3], eidx)
        assert np.array_equal(res[b][1].view(np.uint32), ea.view(np.uint32))


def test_device_path_matches_host(fd, oracle):
    """lsd_map on torch device frames (maps written whole by the kernel, no memsets) equals the host path."""
    torch = pytest.importorskip("torch")
    frames = np.stack([oracle.make_frame("checker", 60 + i, 120, 200, 64) for i in range(2)]
                      + [oracle.make_frame("noise", 70, 120, 200)])
    host = fd.lsd_map(frames)
    dev = torch.from_numpy(frames).cuda()
    out = (torch.full((3, 119, 199), 7.0, device="cuda"), torch.full((3, 119, 199), 7.0, device="cuda"),
           torch.full((3, 119, 199), 7, dtype=torch.uint8, device="cuda"),
           torch.empty((3, 119 * 199), dtype=torch.int32, device="cuda"), torch.empty((3,), dtype=torch.int64, device="cuda"))
    n, a, v, idx, cnt = fd.lsd_map(dev, out=out)
    torch.cuda.synchronize()
    for b in range(3):
        hn, ha, hv, hidx = host[b]
        assert np.array_equal(n[b].cpu().numpy().view(np.uint32), hn.view(np.uint32))
        assert np.array_equal(a[b].cpu().numpy().view(np.uint32), ha.view(np.uint32))
        assert np.array_equal(v[b].cpu().numpy(), hv)
        assert int(cnt[b]) == len(hidx)
        assert np.array_equal(idx[b, :len(hidx)].cpu().numpy(), hidx)


@pytest.mark.parametrize("shape", [(120, 200), (67, 5), (33, 257), (40, 1920)])
def test_pitched_maps(fd, oracle, shape):
    """fd_lsd_map_pitched: the default device maps (rows padded to 16 entries: aligned row stores) and a
    caller pitch (odd on purpose) equal the host path; the padding entries are never written."""
    torch = pytest.importorskip("torch")
    rows, cols = shape
    frames = np.stack([oracle.make_frame("checker", 80 + i, rows, cols, 16) for i in range(2)]
                      + [oracle.make_frame("noise", 90, rows, cols)])
    host = fd.lsd_map(frames)
    dev = torch.from_numpy(frames).cuda()
    mr, mc = rows - 1, cols - 1
    outs = [fd.lsd_map(dev)]
    pitch = mc + 5
    bufs = (torch.full((3, mr, pitch), 7.0, device="cuda"), torch.full((3, mr, pitch), 7.0, device="cuda"),
            torch.full((3, mr, pitch), 7, dtype=torch.uint8, device="cuda"))
    outs.append(fd.lsd_map(dev, out=tuple(t[..., :mc] for t in bufs) + (
        torch.empty((3, mr * mc), dtype=torch.int32, device="cuda"), torch.empty((3,), dtype=torch.int64, device="cuda"))))
    torch.cuda.synchronize()
    assert outs[0][0].stride(1) % 16 == 0 and outs[0][0].stride(1) >= mc
    for n, a, v, idx, cnt in outs:
        for b in range(3):
            hn, ha, hv, hidx = host[b]
            assert np.array_equal(n[b].cpu().numpy().view(np.uint32), hn.view(np.uint32)), b
            assert np.array_equal(a[b].cpu().numpy().view(np.uint32), ha.view(np.uint32)), b
            assert np.array_equal(v[b].cpu().numpy(), hv), b
            assert int(cnt[b]) == len(hidx)
            assert np.array_equal(idx[b, :len(hidx)].cpu().numpy(), hidx), b
    for t, fill in zip(bufs, (7.0, 7.0, 7)):
        assert bool((t[..., mc:] == fill).all())  # padding untouched
    with pytest.raises(Exception):  # a pitch below cols-1 is refused
        bad = torch.empty((3, mr, mc), device="cuda").as_strided((3, mr, mc), (mr * (mc - 1), mc - 1, 1))
        fd.lsd_map(dev, out=(bad, None, None, torch.empty((3, mr * mc), dtype=torch.int32, device="cuda"),
                             torch.empty((3,), dtype=torch.int64, device="cuda")))


def test_config4_batch_spot_check(fd, oracle):
    """BASELINE configs[3] shape (1920x1080 x256, the bench's 64-px checker + noise): the dense maps and
    the valid list of frames 0, 127 and 255 against the oracle, and every frame's count consistent."""
    torch = pytest.importorskip("torch")
    g = torch.Generator(device="cuda")
    g.manual_seed(4243)
    rows, cols, n = 1080, 1920, 256
    r = torch.arange(rows, device="cuda").view(1, rows, 1) // 64
    c = torch.arange(cols, device="cuda").view(1, 1, cols) // 64
    base = torch.where(((r + c) % 2) == 1, 180, 60)
    noise = torch.randint(-10, 11, (n, rows, cols), generator=g, device="cuda", dtype=torch.int32)
    frames = (base + noise).clamp(0, 255).to(torch.uint8)
    nm, am, vm, idx, cnt = fd.lsd_map(frames)  # the bench's layout: row-padded (aligned) maps
    torch.cuda.synchronize()
    assert nm.stride(1) == 1920  # 1919 entries padded to 16
    assert torch.equal(cnt, vm.sum(dim=(1, 2), dtype=torch.int64))
    host = frames.cpu().numpy()
    for b in (0, 127, 255):
        en, ea, ev, eidx = oracle.lsd_map(host[b])
        k = int(cnt[b])
        assert np.array_equal(nm[b].cpu().numpy().view(np.uint32), en.view(np.uint32)), b
        assert np.array_equal(vm[b].cpu().numpy(), ev), b
        assert np.array_equal(am[b].cpu().numpy().view(np.uint32), ea.view(np.uint32)), b
        assert np.array_equal(idx[b, :k].cpu().numpy(), eidx), b
