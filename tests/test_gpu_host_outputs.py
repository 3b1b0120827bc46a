"""Host-output selection calls (fd_points_detect with outputs_on_device = 0): in the raster tie order k_select
writes the features and counts straight into the context's pinned result buffer and mirrors the frames'
status words there (fd_runtime.cpp run_select, SelectArgs::status_host); the reference order copies them
after its pass. Either way the host outputs must equal the device-output call on the same frames, and the
status words fd_ctx_frame_status returns (the cached host copy) must equal the device ones -- for every
detector, a batch with a blank frame (no candidates: the kernel's early exit), a noise frame and a
structured one, and for priors."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}


@pytest.fixture(scope="module")
def fd():
    import feature_detector_amd as fd

    fd.load()
    return fd


def _frames(oracle, rows, cols):
    r, c = np.mgrid[0:rows, 0:cols]
    checker = ((r // 24 + c // 24) % 2 * 120 + 60).astype(np.uint8)
    return np.stack([np.zeros((rows, cols), np.uint8), oracle.make_frame("noise", 77, rows, cols), checker])


@pytest.mark.parametrize("kind", ["harris", "shi_tomasi", "fast"])
@pytest.mark.parametrize("ties", ["raster", "reference"])
def test_host_outputs_equal_device_outputs(fd, oracle, kind, ties):
    torch = pytest.importorskip("torch")
    frames = _frames(oracle, 240, 320)
    ctx = fd.Context(0)
    for rep in range(2):  # (the second call reuses the pinned buffer and the cached status words)
        host = fd.detect_points(kind, frames, 150, 12, THR[kind], ctx=ctx, ties=ties)
        dev = fd.detect_points(kind, torch.from_numpy(frames).cuda(), 150, 12, THR[kind], ctx=ctx, ties=ties)
        torch.cuda.synchronize()
        for b in range(len(frames)):
            assert np.array_equal(host.features(b), dev.features(b)), (kind, ties, rep, b)
            exp, _ = oracle.detect(fd.points.KINDS[kind], frames[b], 12, THR[kind], 150, None,
                                   sort_mode=0 if ties == "reference" else 1)
            assert np.array_equal(host.features(b), exp), (kind, ties, rep, b)
        assert len(host.features(0)) == 0  # the blank frame
        # (FRAME_REDETECTED depends on the emission cut the previous FAST call on the context proposed)
        keep = np.uint32(~fd.points.FRAME_REDETECTED & 0xFFFFFFFF)
        assert np.array_equal(host.frame_flags() & keep, dev.frame_flags() & keep), (host.frame_flags(), dev.frame_flags())
    ctx.close()


def test_host_outputs_with_priors(fd, oracle):
    torch = pytest.importorskip("torch")
    frames = _frames(oracle, 240, 320)
    prior = [np.zeros((0, 2), np.float32), np.array([[100.0, 80.0], [20.5, 30.25]], np.float32),
             np.array([[160.0, 120.0]], np.float32)]
    ctx = fd.Context(0)
    host = fd.detect_points("harris", frames, 100, 15, 30.0, prior=prior, ctx=ctx, ties="raster")
    dev = fd.detect_points("harris", torch.from_numpy(frames).cuda(), 100, 15, 30.0, prior=prior, ctx=ctx, ties="raster")
    torch.cuda.synchronize()
    for b in range(len(frames)):
        assert np.array_equal(host.features(b), dev.features(b)), b
    assert np.array_equal(host.frame_flags(), dev.frame_flags())
    ctx.close()
