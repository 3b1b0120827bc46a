"""GPU: context, stream and status-word semantics of the C ABI (include/fd_hip.h).

* a context's workspace is shared by every call on it: switching streams (host call -> torch stream
  -> another torch stream) must order the new stream after the old one's work, without the caller
  synchronising in between;
* torch inputs pick the context of their own device, and a context on another device is an error;
* device-output calls return plain counts; per-frame flags (ties, guards, out-of-range heatmap
  values) are in fd_ctx_frame_status;
* growing the workspace inside a HIP graph capture fails with a clear error instead of allocating.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}
KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2}


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def test_alternating_streams_on_one_context(fd, oracle):
    torch = pytest.importorskip("torch")
    ctx = fd.Context(0)
    frames = [oracle.make_frame("noise" if i % 2 else "checker", 500 + i, 480, 640) for i in range(6)]
    devs = [torch.from_numpy(f).cuda() for f in frames]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for i, name in enumerate(["harris", "fast", "shi_tomasi", "harris", "fast", "shi_tomasi"]):
        if i % 3 == 0:  # host frames: the context's own stream, synchronous
            r = fd.detect_points(name, frames[i], 200, 20, THR[name], ctx=ctx, ties="raster")
            outs.append((name, i, r.features(0)))
        else:
            s = s1 if i % 3 == 1 else s2
            with torch.cuda.stream(s):
                r = fd.detect_points(name, devs[i][None], 200, 20, THR[name], ctx=ctx, ties="raster")
            outs.append((name, i, r))
    torch.cuda.synchronize()
    for name, i, r in outs:
        got = r if isinstance(r, np.ndarray) else r.features(0)
        exp = oracle.detect(KIND[name], frames[i], 20, THR[name], 200, sort_mode=1)[0]
        np.testing.assert_array_equal(got, exp, err_msg=f"call {i} ({name})")


def test_context_device_mismatch_is_an_error(fd):
    torch = pytest.importorskip("torch")
    from feature_detector_amd.points import _resolve_ctx

    class OtherDevice:  # a context object claiming another GPU
        device = 1

    t = torch.zeros((1, 16, 16), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(ValueError, match="device"):
        _resolve_ctx(OtherDevice(), t)
    assert _resolve_ctx(None, t).device == 0


def test_device_counts_are_plain_and_status_has_flags(fd, oracle):
    torch = pytest.importorskip("torch")
    from feature_detector_amd import superpoint as sp

    heat = np.random.default_rng(3).uniform(0, 1, (2, 120, 160)).astype(np.float32)
    heat[1, 60, 80] = 1.5  # above the declared max_response (1.0)
    dev = torch.from_numpy(heat).cuda()
    ctx = fd.Context(0)
    xy, cnt = sp.nn_select(dev, ctx=ctx)
    st = ctx.frame_status(2)
    c = cnt.cpu().numpy()
    assert (c >= 0).all() and (c <= 241).all()  # no flag bits in the counts
    assert st[1] & fd.points.FRAME_VALUE_RANGE and not st[0] & fd.points.FRAME_VALUE_RANGE
    with pytest.raises(fd.FdError):  # the host-output call reports it as an error
        sp.nn_select(heat, ctx=ctx)


def test_growth_during_capture_fails_cleanly(fd, oracle):
    torch = pytest.importorskip("torch")
    ctx = fd.Context(0)
    img = torch.from_numpy(oracle.make_frame("noise", 1, 240, 320)).cuda()[None]
    out = (torch.empty((1, 201, 2), dtype=torch.float32, device="cuda"),
           torch.empty((1,), dtype=torch.int32, device="cuda"))
    fd.detect_points("harris", img, 200, 20, 30.0, ctx=ctx, out=out, ties="raster")  # sizes the workspace
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    big = torch.zeros((4, 720, 1280), dtype=torch.uint8, device="cuda")
    out4 = (torch.empty((4, 201, 2), dtype=torch.float32, device="cuda"),
            torch.empty((4,), dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    with pytest.raises(fd.FdError, match="captur"):
        with torch.cuda.graph(g):
            fd.detect_points("harris", big, 200, 20, 30.0, ctx=ctx, out=out4, ties="raster")
    torch.cuda.synchronize()
    # the context stays usable afterwards
    r = fd.detect_points("harris", img, 200, 20, 30.0, ctx=ctx, ties="raster")
    torch.cuda.synchronize()
    exp = oracle.detect(0, img[0].cpu().numpy(), 20, 30.0, 200, sort_mode=1)[0]
    np.testing.assert_array_equal(r.features(0), exp)
