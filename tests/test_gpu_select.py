"""GPU: the selection kernel (SelectGoodFeatures, feature_point_detector.cpp:54-88) against the
oracle's restatement across the regimes of its radix descent: no distance test, tiny and huge
cells (LDS grid and global grid), needs that finish inside the first chunk and needs that are never
reached (every candidate visited: many chunks and descents), batches of mixed frames, and repeated
calls of different shapes and kinds (the kernel resets its own counters and histograms).

Every case runs in both tie orders: "raster" (the kernel's total order, against the oracle's stable
order) and "reference" (frames whose scan meets equal responses re-selected in std::sort's order,
against the oracle's std::sort order)."""
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


def _check(fd, oracle, name, frames, need, dist):
    for ties, mode in (("raster", 1), ("reference", 0)):
        res = fd.detect_points(name, frames, need, dist, THR[name], ties=ties)
        for i in range(frames.shape[0]):
            exp = oracle.detect(KIND[name], frames[i], dist, THR[name], need, sort_mode=mode)[0]
            np.testing.assert_array_equal(res.features(i), exp, err_msg=f"{name} frame {i} ties={ties}")


@pytest.mark.parametrize("dist,need", [(0, 50), (1, 500), (3, 200), (20, 200), (60, 100), (254, 10), (255, 10),
                                       (20, 100000)])
@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_select_regimes_against_oracle(fd, oracle, name, dist, need):
    frames = np.stack([oracle.make_frame("noise" if i % 2 == 0 else "checker", 300 + i, 240, 320) for i in range(3)])
    _check(fd, oracle, name, frames, need, dist)


@pytest.mark.parametrize("name", ["harris", "fast"])
def test_batch1_720p(fd, oracle, name):
    # FAST 720p noise consumes ~5k candidates: many sub-chunks of the first chunks
    img = oracle.make_frame("noise", 77, 720, 1280)
    _check(fd, oracle, name, img[None], 200, 20)


def test_repeated_calls_reset_state(fd, oracle):
    a = oracle.make_frame("noise", 5, 200, 300)
    b = oracle.make_frame("checker", 6, 333, 251)
    for _ in range(3):
        for name, img in (("harris", a), ("fast", b), ("shi_tomasi", a), ("harris", b)):
            _check(fd, oracle, name, img[None], 150, 7)
    # batch sizes changing between calls re-lay the control block; it must still read as zero
    for bsz in (4, 1, 7, 2):
        frames = np.stack([oracle.make_frame("noise", 40 + i, 120, 160) for i in range(bsz)])
        _check(fd, oracle, "harris", frames, 60, 5)


@pytest.mark.parametrize("groups", ["1", "3", "64"])
def test_gather_kernel_groups(fd, oracle, groups, monkeypatch):
    # FD_GATHER_GROUPS=1: k_select gathers its first chunk itself; >1: k_gather (own kernel) does
    monkeypatch.setenv("FD_DEBUG_AB", "1")  # (the library reads A/B switches only with it)
    monkeypatch.setenv("FD_GATHER_GROUPS", groups)
    frames = np.stack([oracle.make_frame("noise", 90 + i, 240, 320) for i in range(2)])
    for name in ("harris", "fast"):
        _check(fd, oracle, name, frames, 200, 20)


@pytest.mark.parametrize("seg", ["0", "1"])
def test_sorted_segment_lists_toggle(fd, oracle, seg, monkeypatch):
    # FD_SEG_LISTS=1 (default below a megapixel): each candidate-kernel workgroup writes its list
    # segment sorted by level-0 bin and k_select reads only the segments' prefixes for its first
    # chunk; tiles that overflow their staging (dense FAST) mark the frame and k_select scans it
    monkeypatch.setenv("FD_DEBUG_AB", "1")  # (the library reads A/B switches only with it)
    monkeypatch.setenv("FD_SEG_LISTS", seg)
    for shape, bsz in (((480, 640), 1), ((240, 320), 3), ((61, 77), 2), ((700, 1000), 1)):
        frames = np.stack([oracle.make_frame("noise" if i % 2 == 0 else "checker", 700 + i, *shape) for i in range(bsz)])
        for name, dist, need in (("harris", 20, 200), ("shi_tomasi", 3, 800), ("fast", 20, 200), ("harris", 0, 50)):
            _check(fd, oracle, name, frames, need, dist)


@pytest.mark.parametrize("rows,cols,dist", [(24, 32760, 3), (24, 40000, 20), (20, 65400, 100), (33000, 24, 20)])
@pytest.mark.parametrize("name", ["harris", "fast"])
def test_wide_frames_grid_sentinels(fd, oracle, name, rows, cols, dist):
    # The greedy's occupancy grid marks empty cells 0x7FFF7FFF (a position that fails the packed distance
    # test by itself) only while rows, cols + 3d < 2^15; wider frames keep 0xFFFFFFFF with explicit
    # checks, in the packed-halves test (+ 3d < 2^16) or the plain one (the 65400-column case).
    img = oracle.make_frame("noise", 910 + cols % 97, rows, cols)
    _check(fd, oracle, name, img[None], 400, dist)
