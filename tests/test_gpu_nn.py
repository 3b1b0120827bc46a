"""GPU parity of the SuperPoint post-processing (fd_nn_select / fd_nn_descriptors)
against the CPU oracle (nn_feature_point_detector.cpp:59-73, 128-155, 163-193), and the random-weight
SuperPoint network end to end (network outputs checked through the oracle on the same tensors).

Bar: bit-exact features (multimap order: response descending, ties by raster index descending) and
descriptor values. The network's weights are seeded random (no trained model offline): its
keypoints are not comparable with the reference's ("parity unpinned" for the network itself).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sp():
    import feature_detector_amd as fd
    from feature_detector_amd import superpoint

    fd.load()
    return superpoint


def features(xy, cnt, b):
    xy = xy if isinstance(xy, np.ndarray) else xy.cpu().numpy()
    n = int(cnt[b]) if isinstance(cnt, np.ndarray) else int(cnt[b].item())
    return xy[b, :n]


@pytest.mark.parametrize("border,dist,maxf,thr", [(3, 15, 240, 0.1), (0, 4, 300, 0.5), (5, 0, 50, 0.3),
                                                  (3, 15, 1, 0.1), (3, 40, 240, 0.2), (2, 1, 5000, 0.05)])
def test_nn_select_matches_oracle(sp, oracle, border, dist, maxf, thr):
    rng = np.random.default_rng(dist * 7 + maxf)
    heat = np.stack([(np.round(rng.random((120, 160)) * 32) / 32).astype(np.float32),  # many ties
                     rng.random((120, 160)).astype(np.float32),
                     np.zeros((120, 160), np.float32)])
    o = sp.Options(kInvalidBoundary=border, kMinFeatureDistance=dist, kMaxNumberOfDetectedFeatures=maxf,
                   kMinResponse=thr)
    xy, cnt = sp.nn_select(heat, o)
    for b in range(3):
        exp = oracle.nn_select(heat[b], border, dist, maxf, thr)
        assert np.array_equal(features(xy, cnt, b), exp), b


def test_nn_select_priors(sp, oracle):
    rng = np.random.default_rng(11)
    heat = rng.random((2, 96, 128)).astype(np.float32)
    prior = [np.array([(10.5, 20.7), (100.0, 50.0), (-4.0, 3.0)], np.float32), np.zeros((0, 2), np.float32)]
    o = sp.Options(kMaxNumberOfDetectedFeatures=40)
    xy, cnt = sp.nn_select(heat, o, prior)
    for b in range(2):
        exp = oracle.nn_select(heat[b], 3, 15, 40, 0.1, prior[b] if len(prior[b]) else None)
        assert np.array_equal(features(xy, cnt, b), exp)


def test_nn_descriptors_matches_oracle(sp, oracle):
    rng = np.random.default_rng(3)
    m = rng.standard_normal((2, 256, 15, 20)).astype(np.float32)
    xy = np.stack([rng.uniform(-10, 170, (33, 2)), rng.uniform(0, 160, (33, 2))]).astype(np.float32)
    xy[0, :5] = np.round(xy[0, :5])
    counts = np.array([33, 20], np.int32)
    got = sp.nn_descriptors(m, xy, counts)
    for b in range(2):
        exp = oracle.nn_descriptors(m[b], xy[b, :counts[b]])
        assert np.array_equal(got[b, :counts[b]].view(np.uint32), exp.view(np.uint32))
        assert not got[b, counts[b]:].any()


@pytest.mark.parametrize("rows,cols,n", [(240, 320, 3), (480, 640, 4)])  # 480x640: BASELINE configs[4]'s shape
def test_superpoint_end_to_end_device(sp, oracle, rows, cols, n):
    """Random-weight SuperPoint on device frames: GPU selection + descriptors equal the oracle's
    post-processing of the very same network outputs."""
    torch = pytest.importorskip("torch")
    det = sp.SuperPointDetector(sp.Options(kComputeDescriptors=True, kMaxImageRows=rows, kMaxImageCols=cols))
    assert det.Initialize()
    frames = torch.from_numpy(np.stack([oracle.make_frame("noise", 900 + i, rows, cols) for i in range(n)])).cuda()
    xy2, cnt2, d2 = det.DetectGoodFeaturesWithDescriptor(frames)
    assert tuple(xy2.shape) == (n, 241, 2) and tuple(d2.shape) == (n, 241, 256)
    # the same post-processing on one network run (MIOpen may pick different algorithms per call)
    heat, desc = det.InferenceSession(frames)
    xy, cnt = sp.nn_select(heat, det.options())
    d = sp.nn_descriptors(desc, xy, cnt)
    torch.cuda.synchronize()
    heat_h, desc_h = heat.float().cpu().numpy(), desc.float().cpu().numpy()
    cnt_h = cnt.cpu().numpy()
    assert cnt_h.min() > 0
    for b in range(n):
        exp = oracle.nn_select(heat_h[b], 3, 15, 240, 0.1)
        got = features(xy, cnt, b)
        assert np.array_equal(got, exp)
        ed = oracle.nn_descriptors(desc_h[b], got)
        assert np.array_equal(d[b, :cnt_h[b]].cpu().numpy().view(np.uint32), ed.view(np.uint32))


def test_nn_select_key_range(sp, oracle):
    """Probabilities (max_response 1, fine keys) and an unbounded map give the same features; a value
    above the declared maximum fails the call instead of being misordered."""
    import feature_detector_amd as fd

    rng = np.random.default_rng(21)
    heat = (rng.random((2, 100, 140)) ** 3).astype(np.float32)
    o = sp.Options(kMaxNumberOfDetectedFeatures=120, kMinFeatureDistance=6)
    a, ca = sp.nn_select(heat, o)
    b, cb = sp.nn_select(heat, o, max_response=float("inf"))
    assert np.array_equal(ca, cb) and np.array_equal(a, b)
    for f in range(2):
        assert np.array_equal(features(a, ca, f), oracle.nn_select(heat[f], 3, 6, 120, 0.1))
    bad = heat.copy()
    bad[1, 50, 70] = 1.5
    with pytest.raises(fd.FdError):
        sp.nn_select(bad, o)
    c, cc = sp.nn_select(bad, o, max_response=float("inf"))
    assert np.array_equal(features(c, cc, 1), oracle.nn_select(bad[1], 3, 6, 120, 0.1))
    # the failed call left the control block clean for the next one
    d, cd = sp.nn_select(heat, o)
    assert np.array_equal(cd, ca) and np.array_equal(d, a)


def test_nn_descriptors_channels_last_in_place(sp, oracle):
    """A channels-last device map (the network's layout) is read in place (FD_MAP_NHWC) and gives the
    same values as the reference's per-channel planes."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(8)
    m = rng.standard_normal((2, 256, 12, 16)).astype(np.float32)
    xy = rng.uniform(-4, 130, (2, 40, 2)).astype(np.float32)
    cnt = torch.tensor([40, 17], dtype=torch.int32, device="cuda")
    md = torch.from_numpy(m).cuda()
    xyd = torch.from_numpy(xy).cuda()
    a = sp.nn_descriptors(md, xyd, cnt)
    b = sp.nn_descriptors(md.contiguous(memory_format=torch.channels_last), xyd, cnt)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    for f, n in ((0, 40), (1, 17)):
        exp = oracle.nn_descriptors(m[f], xy[f, :n])
        assert np.array_equal(b[f, :n].cpu().numpy().view(np.uint32), exp.view(np.uint32))


# ------------------------------------------------------------------ keypoint-list models (kSuperpointNms / kDiskNms)
def random_lists(rng, b, k, rows, cols, levels=16):
    """Keypoint lists with many equal scores and some repeated pixels."""
    kp = np.stack([rng.integers(0, cols, (b, k)), rng.integers(0, rows, (b, k))], -1).astype(np.int64)
    kp[:, 1::7] = kp[:, 0::7][:, :kp[:, 1::7].shape[1]]  # repeats
    sc = (rng.integers(0, levels, (b, k)) / levels).astype(np.float32)
    return kp, sc


@pytest.mark.parametrize("border,dist,maxf", [(3, 15, 240), (0, 4, 300), (5, 0, 50), (3, 6, 1), (2, 1, 5000)])
def test_nn_select_list_matches_oracle(sp, oracle, border, dist, maxf):
    rng = np.random.default_rng(border * 31 + dist)
    rows, cols, b, k = 120, 160, 3, 2000
    kp, sc = random_lists(rng, b, k, rows, cols)
    counts = np.array([k, 700, 0], np.int64)
    desc = rng.standard_normal((b, k, 64)).astype(np.float32)
    prior = [np.array([(10.5, 20.7), (100.0, 50.0)], np.float32), np.zeros((0, 2), np.float32),
             np.array([(5.0, 5.0)], np.float32)]
    o = sp.Options(kInvalidBoundary=border, kMinFeatureDistance=dist, kMaxNumberOfDetectedFeatures=maxf)
    for pr in (None, prior):
        xy, cnt, d = sp.nn_select_list(kp, sc, rows, cols, counts, o, pr, desc)
        for f in range(b):
            p = None if pr is None or len(pr[f]) == 0 else pr[f]
            exp, idx = oracle.nn_select_list(kp[f, :counts[f]], sc[f, :counts[f]], rows, cols, border, dist, maxf, p)
            assert np.array_equal(features(xy, cnt, f), exp), (f, pr is None)
            assert np.array_equal(d[f, :cnt[f]], desc[f, idx])


def test_nn_select_list_device_and_checks(sp, oracle):
    torch = pytest.importorskip("torch")
    import feature_detector_amd as fd

    rng = np.random.default_rng(5)
    rows, cols, b, k = 96, 128, 2, 900
    kp, sc = random_lists(rng, b, k, rows, cols, levels=1000)
    desc = rng.standard_normal((b, k, 32)).astype(np.float32)
    o = sp.Options(kMaxNumberOfDetectedFeatures=100, kMinFeatureDistance=5)
    xy, cnt, d = sp.nn_select_list(torch.from_numpy(kp).cuda(), torch.from_numpy(sc).cuda(), rows, cols, None, o,
                                   None, torch.from_numpy(desc).cuda())
    torch.cuda.synchronize()
    for f in range(b):
        exp, idx = oracle.nn_select_list(kp[f], sc[f], rows, cols, 3, 5, 100)
        assert np.array_equal(features(xy, cnt, f), exp)
        assert np.array_equal(d[f, :len(idx)].cpu().numpy(), desc[f, idx])
    bad = kp.copy()
    bad[1, 3] = (cols, 0)  # outside the frame
    with pytest.raises(fd.FdError):
        sp.nn_select_list(bad, sc, rows, cols, None, o)
    xy2, cnt2, _ = sp.nn_select_list(kp, sc, rows, cols, None, o)  # the context is clean after the refusal
    assert np.array_equal(features(xy2, cnt2, 0), features(xy, cnt, 0))


@pytest.mark.parametrize("model", ["kSuperpointHeatmap", "kSuperpointNms", "kDiskHeatmap", "kDiskNms"])
def test_model_types_end_to_end(sp, oracle, model):
    """Each ModelType on device frames (random weights): the GPU post-processing equals the oracle's on
    the same network outputs; heatmap models also describe the prior features (all_pixel_uv)."""
    torch = pytest.importorskip("torch")
    rows, cols, n = 96, 128, 2
    o = sp.Options(kModelType=model, kMaxImageRows=rows, kMaxImageCols=cols, kMaxNumberOfDetectedFeatures=60)
    det = sp.NNFeaturePointDetector(o, top_k=400)
    assert det.Initialize()
    frames = torch.from_numpy(np.stack([oracle.make_frame("noise", 70 + i, rows, cols) for i in range(n)])).cuda()
    prior = [np.array([(20.0, 30.0), (64.5, 40.2)], np.float32), np.zeros((0, 2), np.float32)]
    out = det.InferenceSession(frames)
    dim = 128 if "Disk" in model else 256
    if model.endswith("Nms"):
        kp, sc, dl = (t.float().cpu().numpy() if t.dtype != torch.int64 else t.cpu().numpy() for t in out)
        xy, cnt, d = sp.nn_select_list(out[0], out[1], rows, cols, None, o, prior, out[2])
        torch.cuda.synchronize()
        assert tuple(d.shape) == (n, 61, dim)
        for f in range(n):
            p = prior[f] if len(prior[f]) else None
            exp, idx = oracle.nn_select_list(kp[f], sc[f], rows, cols, 3, 15, 60, p)
            assert len(exp) > 0
            assert np.array_equal(features(xy, cnt, f), exp)
            assert np.array_equal(d[f, :len(idx)].cpu().numpy(), dl[f, idx])
    else:
        heat, desc = out
        heat_h, desc_h = heat.float().cpu().numpy(), desc.float().cpu().numpy()
        assert desc_h.shape[1] == dim
        xy, cnt = sp.nn_select(heat, o, prior)
        d = sp.nn_descriptors(desc, xy, cnt)
        torch.cuda.synchronize()
        for f in range(n):
            p = prior[f] if len(prior[f]) else None
            exp = oracle.nn_select(heat_h[f], 3, 15, 60, 0.1, p)
            assert len(exp) > 0
            got = features(xy, cnt, f)
            assert np.array_equal(got, exp)
            assert np.array_equal(d[f, :len(got)].cpu().numpy().view(np.uint32),
                                  oracle.nn_descriptors(desc_h[f], got).view(np.uint32))
    res = det.DetectGoodFeaturesWithDescriptor(frames, prior)
    xy_r, cnt_r, d_r = res
    torch.cuda.synchronize()
    assert tuple(d_r.shape)[2] == dim and int(cnt_r.min()) > 0
    if model.endswith("Nms"):
        assert res.prior_descriptors is None
    else:  # descriptors of the incoming features too (all_pixel_uv), rows 0.. of each frame
        pd = res.prior_descriptors.cpu().numpy()
        assert pd.shape == (n, 2, dim) and not pd[1].any() and np.abs(pd[0]).sum() > 0
        exp = oracle.nn_descriptors(desc_h[0], prior[0])
        pxy = torch.from_numpy(np.stack([prior[0], np.zeros((2, 2), np.float32)])).cuda()
        got = sp.nn_descriptors(desc, pxy, torch.tensor([2, 0], dtype=torch.int32, device="cuda"))
        assert np.array_equal(got[0].cpu().numpy().view(np.uint32), exp.view(np.uint32))


def _reference_forward(net, x):
    """SuperPointNet.forward with PyTorch's own modules only (biased convolution, ReLU, MaxPool2d)."""
    import torch

    r, p = net.relu, net.pool
    x = p(r(net.conv1b(r(net.conv1a(x)))))
    x = p(r(net.conv2b(r(net.conv2a(x)))))
    x = p(r(net.conv3b(r(net.conv3a(x)))))
    x = r(net.conv4b(r(net.conv4a(x))))
    semi = net.convPb(r(net.convPa(x))).float()
    heat = torch.nn.functional.pixel_shuffle(torch.softmax(semi, dim=1)[:, :-1], 8)[:, 0]
    desc = net.convDb(r(net.convDa(x))).float()
    return heat, desc / desc.norm(dim=1, keepdim=True).clamp_min(1e-12)


@pytest.mark.gpu
def test_conv1_bias_relu_matches_torch(sp):
    """fd_nn_conv3x3_c1 (first layer: 1 input channel, 3x3, padding 1, + bias + ReLU) against PyTorch's
    float32 convolution of the same fp16 tensors: within two fp16 rounding steps (the kernel rounds the
    convolution to half, then the biased sum), on frame edges and ragged sizes; argument checks."""
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    for n, h, w, c in ((2, 17, 23, 64), (1, 480, 640, 64), (3, 8, 9, 8), (1, 5, 300, 256)):
        x = torch.rand((n, 1, h, w), generator=g, device="cuda").half()
        wt = (torch.randn((c, 1, 3, 3), generator=g, device="cuda") * 0.5).half()
        b = (torch.randn(c, generator=g, device="cuda") * 0.2).half()
        got = sp.conv1_bias_relu(x.contiguous(memory_format=torch.channels_last), wt, b)
        assert got.is_contiguous(memory_format=torch.channels_last)
        conv = torch.nn.functional.conv2d(x.float(), wt.float(), None, 1, 1)
        ref = torch.relu(conv + b.float().view(1, -1, 1, 1))
        err = (got.float() - ref).abs()
        tol = (conv.abs() + ref.abs()) * 2.0 ** -10 + 2.0 ** -14  # one half rounding of each sum (+ margin)
        assert bool((err <= tol).all()), (n, h, w, c, err.max().item())
        assert bool((got >= 0).all())
    x = torch.zeros((1, 2, 4, 4), device="cuda", dtype=torch.float16)
    with pytest.raises(ValueError):
        sp.conv1_bias_relu(x, torch.zeros((8, 1, 3, 3), device="cuda", dtype=torch.float16),
                           torch.zeros(8, device="cuda", dtype=torch.float16))  # two input channels
    x = torch.zeros((1, 1, 4, 4), device="cuda", dtype=torch.float16)
    with pytest.raises(ValueError):
        sp.conv1_bias_relu(x, torch.zeros((8, 1, 3, 3), device="cuda", dtype=torch.float16),
                           torch.zeros(4, device="cuda", dtype=torch.float16))  # short bias
    import ctypes
    from feature_detector_amd import _lib
    ctx = sp._resolve_ctx(None, x)
    rc = _lib.load().fd_nn_conv3x3_c1(ctx.ptr, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                       ctypes.c_void_p(x.data_ptr()), 12, ctypes.c_void_p(x.data_ptr()), 1, 4, 4)
    assert rc != 0  # 12 channels: not a supported group count


@pytest.mark.gpu
def test_conv64_bias_relu_matches_torch(sp):
    """fd_nn_conv3x3_c64 (64 -> 64 / 128 channels, 3x3, padding 1, + bias + ReLU, with and without the 2x2 max pool,
    on the matrix cores) against PyTorch's float32 convolution of the same fp16 tensors, within one fp16
    rounding of the convolution and one of the biased sum; ragged tiles (sizes not multiples of the 4 x 64
    tile), a 640x480 frame, and argument checks."""
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    for n, h, w, co in ((2, 8, 64, 64), (1, 6, 130, 128), (3, 10, 18, 64), (1, 480, 640, 64), (2, 120, 160, 128)):
        x = torch.rand((n, 64, h, w), generator=g, device="cuda").half().contiguous(memory_format=torch.channels_last)
        wt = (torch.randn((co, 64, 3, 3), generator=g, device="cuda") * 0.06).half()
        b = (torch.randn(co, generator=g, device="cuda") * 0.2).half()
        conv = torch.nn.functional.conv2d(x.float(), wt.float(), None, 1, 1)
        ref = torch.relu(conv + b.float().view(1, -1, 1, 1))
        tol = (conv.abs() + ref.abs()) * 2.0 ** -10 + 2.0 ** -14
        got = sp.conv64_bias_relu(x, wt, b)
        assert got.is_contiguous(memory_format=torch.channels_last)
        err = (got.float() - ref).abs()
        assert bool((err <= tol).all()), (n, h, w, err.max().item())
        gp = sp.conv64_bias_relu(x, wt, b, pool=True)
        refp = torch.nn.functional.max_pool2d(ref, 2, 2)
        tolp = torch.nn.functional.max_pool2d(tol, 2, 2)
        assert tuple(gp.shape) == (n, co, h // 2, w // 2)
        assert bool(((gp.float() - refp).abs() <= tolp).all()), (n, h, w, (gp.float() - refp).abs().max().item())
    x = torch.zeros((1, 64, 5, 8), device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    wt = torch.zeros((64, 64, 3, 3), device="cuda", dtype=torch.float16)
    with pytest.raises(ValueError):
        sp.conv64_bias_relu(x, wt, torch.zeros(64, device="cuda", dtype=torch.float16), pool=True)  # odd H
    with pytest.raises(ValueError):
        sp.conv64_bias_relu(x.contiguous(), wt, torch.zeros(64, device="cuda", dtype=torch.float16))  # NCHW
    with pytest.raises(ValueError):
        sp.conv64_bias_relu(x, wt, torch.zeros(32, device="cuda", dtype=torch.float16))  # short bias


@pytest.mark.gpu
def test_bias_relu_matches_torch(sp):
    """fd_nn_bias_relu (bias + ReLU, and + 2x2 max pool, on channels-last fp16) equals PyTorch's separate
    half-precision ops bit for bit. The fused SuperPoint forward runs the convolutions without their bias,
    which is not bit-identical to PyTorch's biased convolution (MIOpen may apply the bias before the
    fp16 rounding of the convolution's output), so the network is compared within fp16 tolerance
    (the network has seeded random weights: no reference output exists for it)."""
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for c in (8, 64, 256):
        x = (torch.randn(3, c, 34, 50, generator=g, device="cuda") * 8).half().contiguous(memory_format=torch.channels_last)
        b = (torch.randn(c, generator=g, device="cuda") * 4).half()
        ref = torch.relu(x + b.view(1, -1, 1, 1))
        got = sp.bias_relu(x, b)
        assert torch.equal(got, ref), c
        refp = torch.nn.functional.max_pool2d(ref, 2, 2)
        assert torch.equal(sp.bias_relu(x, b, pool=True), refp), c
        inplace = x.clone(memory_format=torch.channels_last)
        sp.bias_relu(inplace, b, out=inplace)
        assert torch.equal(inplace, ref), c
    with pytest.raises(ValueError):
        sp.bias_relu(torch.zeros(1, 8, 4, 4, device="cuda"), torch.zeros(8, device="cuda"))  # fp32, not fp16
    x8 = torch.zeros(1, 16, 4, 4, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    with pytest.raises(ValueError):
        sp.bias_relu(x8, torch.zeros(8, device="cuda", dtype=torch.float16))  # short bias
    with pytest.raises(ValueError):
        sp.bias_relu(x8, torch.zeros(16, device="cuda", dtype=torch.float16), pool=True, out=x8)  # out not pooled
    import ctypes
    from feature_detector_amd import _lib
    ctx = sp._resolve_ctx(None, x8)
    b16 = torch.zeros(16, device="cuda", dtype=torch.float16)
    rc = _lib.load().fd_nn_bias_relu(ctx.ptr, ctypes.c_void_p(x8.data_ptr()), ctypes.c_void_p(b16.data_ptr()), 8,
                                      ctypes.c_void_p(x8.data_ptr()), 1, 4, 4, 16, 0)
    assert rc != 0  # the C ABI refuses a bias length that is not the channel count
    net = sp.build_net(0).cuda().eval().half().to(memory_format=torch.channels_last)
    frames = torch.randint(0, 256, (2, 1, 96, 128), generator=g, device="cuda", dtype=torch.int32)
    x = (frames.half() / 255.0).contiguous(memory_format=torch.channels_last)
    with torch.inference_mode():
        heat, desc = net(x)
        rheat, rdesc = _reference_forward(net, x)
    dh = (heat - rheat).abs().max().item()
    dd = (desc - rdesc).abs().max().item()
    print(f"fused vs module forward: max |d heat| {dh:.3g} (max heat {rheat.max().item():.3g}), max |d desc| {dd:.3g}")
    assert torch.allclose(heat, rheat, rtol=2e-2, atol=2e-3) and torch.allclose(desc, rdesc, rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
def test_heads_match_torch(sp):
    """fd_nn_heat_softmax (softmax over 65 channels, dustbin dropped, pixel_shuffle(8)) and
    fd_nn_desc_normalize (per-cell L2 normalisation) on channels-last fp16 logits against PyTorch's float32
    ops on the same values: within float rounding (the sums run in another order); ragged cell counts
    (the 32-cell groups of the heat kernel), a 640x480 batch's 1/8 maps, extreme logits; the model's own
    head tensors take the fused path; argument checks."""
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(31)
    for n, hc, wc in ((1, 1, 1), (2, 3, 33), (3, 7, 64), (64, 60, 80)):
        semi = (torch.randn((n, 65, hc, wc), generator=g, device="cuda") * 6).half().contiguous(memory_format=torch.channels_last)
        ref = torch.nn.functional.pixel_shuffle(torch.softmax(semi.float(), dim=1)[:, :-1], 8)[:, 0]
        got = sp.heat_softmax(semi)
        assert tuple(got.shape) == (n, 8 * hc, 8 * wc) and got.dtype == torch.float32
        assert torch.allclose(got, ref, rtol=1e-5, atol=1e-7), (n, hc, wc, (got - ref).abs().max().item())
        hb = (torch.randn(65, generator=g, device="cuda") * 4).half()  # convPb's bias, added in half first
        refb = torch.nn.functional.pixel_shuffle(torch.softmax((semi + hb.view(1, -1, 1, 1)).float(), dim=1)[:, :-1], 8)[:, 0]
        assert torch.allclose(sp.heat_softmax(semi, hb), refb, rtol=1e-5, atol=1e-7), (n, hc, wc)
        for c in (8, 64, 128, 256, 1024):
            d = (torch.randn((n, c, hc, wc), generator=g, device="cuda") * 3).half().contiguous(memory_format=torch.channels_last)
            df = d.float()
            refd = df / df.norm(dim=1, keepdim=True).clamp_min(1e-12)
            gotd = sp.desc_normalize(d)
            assert gotd.is_contiguous(memory_format=torch.channels_last) and gotd.dtype == torch.float32
            assert torch.allclose(gotd, refd, rtol=1e-5, atol=1e-7), (n, c, (gotd - refd).abs().max().item())
            db = (torch.randn(c, generator=g, device="cuda") * 2).half()
            dbf = (d + db.view(1, -1, 1, 1)).float()
            refdb = dbf / dbf.norm(dim=1, keepdim=True).clamp_min(1e-12)
            assert torch.allclose(sp.desc_normalize(d, db), refdb, rtol=1e-5, atol=1e-7), (n, c)
    big = torch.full((1, 65, 2, 2), 60000.0, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    big[:, 3] = -60000.0
    assert torch.allclose(sp.heat_softmax(big), torch.nn.functional.pixel_shuffle(
        torch.softmax(big.float(), dim=1)[:, :-1], 8)[:, 0], rtol=1e-5, atol=1e-7)
    zero = torch.zeros((1, 16, 2, 3), device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    assert torch.equal(sp.desc_normalize(zero), torch.zeros((1, 16, 2, 3), device="cuda"))
    with pytest.raises(ValueError):
        sp.heat_softmax(torch.zeros((1, 65, 2, 2), device="cuda", dtype=torch.float16))  # NCHW
    with pytest.raises(ValueError):
        sp.desc_normalize(torch.zeros((1, 12, 2, 2), device="cuda", dtype=torch.float16).contiguous(
            memory_format=torch.channels_last))  # 12 channels
    net = sp.build_net(0).cuda().eval().half().to(memory_format=torch.channels_last)
    x = (torch.rand((2, 1, 96, 128), generator=g, device="cuda")).half().contiguous(memory_format=torch.channels_last)
    with torch.inference_mode():
        y = net.cbr(net.conv4b, net.cbr(net.conv4a, torch.zeros((2, 128, 12, 16), device="cuda", dtype=torch.float16)
                                         .contiguous(memory_format=torch.channels_last)))
        xp, xd = net.cbr(net.convPa, y), net.cbr(net.convDa, y)
        assert net.fused_heads(torch.nn.functional.conv2d(xp, net.convPb.weight), torch.nn.functional.conv2d(xd, net.convDb.weight))
        heat, desc = net(x)
        rheat, rdesc = _reference_forward(net, x)
    assert tuple(heat.shape) == (2, 96, 128) and tuple(desc.shape) == (2, 256, 12, 16)
    assert torch.allclose(heat, rheat, rtol=2e-2, atol=2e-3) and torch.allclose(desc, rdesc, rtol=2e-2, atol=2e-3)
