"""FAST's adaptive emission cut (raster tie order; PointsArgs::emit_cut).

The per-pixel kernel emits only candidates at or above a response cut that the previous FAST call's
selection proposed; a frame whose greedy scan runs out of emitted keys with candidates left below the cut
is detected and selected again in the same call, without the cut (FRAME_REDETECTED). The bar is the same as
everywhere: the features equal the oracle's SelectGoodFeatures (stable raster order, sort_mode 1) bit for
bit, whether or not a frame was redetected -- including inside a captured graph, where the cut words
alternate between the captured calls."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THR = 10.0


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def _expect(oracle, frames, need=200, dist=20):
    return [oracle.detect(2, f, dist, THR, need, None, sort_mode=1)[0] for f in frames]


def test_cut_then_sparse_frame_redetected(fd, oracle, image_png):
    """Noise frames first (their selections propose a high cut), then frames whose candidates all lie
    below it: they must be redetected and still equal the oracle; then noise again (no redetection once the
    cut has adapted)."""
    ctx = fd.Context(0)
    noise = np.stack([oracle.make_frame("noise", 3300 + i, 720, 1280) for i in range(4)])
    exp_noise = _expect(oracle, noise)
    for _ in range(3):  # the cut settles on the noise statistics
        res = fd.detect_points("fast", noise, 200, 20, THR, ctx=ctx, ties="raster")
        for b in range(len(noise)):
            assert np.array_equal(res.features(b), exp_noise[b]), b
    st = res.frame_flags()
    assert not (st & fd.points.FRAME_REDETECTED).any(), st
    # image.png (752x480, 962 candidates above 10, responses mostly below the noise frames' top bins)
    res = fd.detect_points("fast", image_png, 200, 20, THR, ctx=ctx, ties="raster")
    assert np.array_equal(res.features(0), _expect(oracle, [image_png])[0])
    assert res.frame_flags()[0] & fd.points.FRAME_REDETECTED
    # a mixed batch: the noise cut again, then sparse and noise frames side by side
    for _ in range(2):
        fd.detect_points("fast", noise, 200, 20, THR, ctx=ctx, ties="raster")
    r, c = np.mgrid[0:720, 0:1280]
    smooth = ((r // 8 + c // 8) % 7 * 9 + 40).astype(np.uint8)  # few, weak corners
    mixed = np.stack([noise[0], smooth, noise[1], smooth[::-1].copy()])
    res = fd.detect_points("fast", mixed, 200, 20, THR, ctx=ctx, ties="raster")
    exp = _expect(oracle, mixed)
    for b in range(len(mixed)):
        assert np.array_equal(res.features(b), exp[b]), b
    ctx.close()


def test_cut_device_outputs_and_graph(fd, oracle):
    """Device frames and outputs (asynchronous), then the same calls captured in a hipGraph (two calls per
    graph, so the cut words alternate inside it) and replayed: every replay equals the oracle, also when
    the second captured call's frames are sparse enough to be redetected."""
    torch = pytest.importorskip("torch")
    ctx = fd.Context(0)
    a = np.stack([oracle.make_frame("noise", 4400 + i, 720, 1280) for i in range(3)])
    r, c = np.mgrid[0:720, 0:1280]
    b = np.stack([((r // 8 + c // 8) % 7 * 9 + 40 + i).astype(np.uint8) for i in range(3)])
    exp_a, exp_b = _expect(oracle, a), _expect(oracle, b)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    outs = [(torch.empty((3, 201, 2), dtype=torch.float32, device="cuda"), torch.empty((3,), dtype=torch.int32, device="cuda"),
             torch.empty((3,), dtype=torch.int32, device="cuda")) for _ in range(2)]

    def two_calls():
        fd.detect_points("fast", da, 200, 20, THR, ctx=ctx, ties="raster", out=outs[0])
        fd.detect_points("fast", db, 200, 20, THR, ctx=ctx, ties="raster", out=outs[1])

    def check():
        torch.cuda.synchronize()
        for (xy, cnt, st), exp in ((outs[0], exp_a), (outs[1], exp_b)):
            for k in range(3):
                assert np.array_equal(xy[k, :int(cnt[k])].cpu().numpy(), exp[k]), k
            assert not (st.cpu().numpy().astype(np.uint32) & np.uint32(fd.points.FRAME_GUARD)).any()

    for _ in range(3):
        two_calls()
        check()
    ctx.reserve(fd.FD_FAST, 3, 720, 1280)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        two_calls()
    for _ in range(4):
        for xy, cnt, st in outs:
            xy.zero_()
            cnt.zero_()
        g.replay()
        check()
    del g
    ctx.close()
