"""oracle.select (SelectGoodFeatures over given candidates, the fd_points_select checker) agrees with
oracle.detect's own selection on the built-in detectors' raster-pushed candidate lists."""
import numpy as np
import pytest


@pytest.mark.parametrize("kind,thr", [(0, 30.0), (1, 40.0), (2, 10.0)])
def test_select_matches_detect(oracle, kind, thr):
    img = oracle.make_frame("checker", 17, 160, 200)
    prior = np.array([[30.0, 40.0], [150.5, 99.9]], np.float32)
    mask = np.ones(img.shape, np.int32)
    for fx, fy in prior:
        r0, c0 = int(fy), int(fx)
        mask[max(r0 - 6, 0):r0 + 7, max(c0 - 6, 0):c0 + 7] = 0
    if kind == 2:
        r, x, y = oracle.fast_candidates(img, thr, mask)
    else:
        r, x, y = oracle.nms(oracle.response_map(img, kind, thr, mask), thr)
    for sm in (0, 1):
        got, (sr, _, _) = oracle.select(r, x, y, 160, 200, 6, 60, prior, sort_mode=sm, sorted_out=True)
        exp, cands = oracle.detect(kind, img, 6, thr, 60, prior, sort_mode=sm)
        assert np.array_equal(got, exp)
        assert np.array_equal(sr, cands[0])


def test_select_duplicates_and_negative_distance(oracle):
    r = np.array([5, 5, 3, 9, 9], np.float32)
    x = np.array([4, 4, 6, 1, 1], np.int32)
    y = np.array([2, 2, 2, 0, 0], np.int32)
    # d = 0: a pixel's box is itself, the second copy is masked; d < 0: no boxes at all (:77-78)
    assert oracle.select(r, x, y, 10, 10, 0, 10).tolist() == [[1, 0], [4, 2], [6, 2]]
    assert oracle.select(r, x, y, 10, 10, -1, 10).tolist() == [[1, 0], [1, 0], [4, 2], [4, 2], [6, 2]]
    assert oracle.select(r, x, y, 10, 10, 2, 10).tolist() == [[1, 0], [4, 2]]


@pytest.mark.parametrize("n", [17, 100, 1000, 5000, 20000])
@pytest.mark.parametrize("front", [True, False])
def test_introsort_restatement_on_killer_inputs(oracle, n, front):
    """libstdc++ 11's std::sort restated (oracle/fd_oracle_introsort.cpp: introsort loop, median of three,
    unguarded partition, depth limit 2 floor(log2 n) -> __make_heap + __sort_heap, final insertion sort)
    gives std::sort's own permutation on McIlroy-adversary inputs, which reach the heapsort fallback and
    carry a run of equal responses into the heapsorted range: the fallback's order of ties is pinned to
    the real library here, and the GPU emulation (fd_select_ref.hip ref_heapsort) is checked against it."""
    r = oracle.introsort_killer(n, front)
    perm, stats = oracle.std_sort_restated(r)
    assert np.array_equal(perm, oracle.std_sort_perm(r))
    if n >= 40:
        assert stats[0] >= 1  # the depth limit was reached
        if front:
            assert stats[1] == 0 and stats[2] > n // 2  # ... in the range the greedy visits first
        srt = r[perm]
        assert (srt[1:] == srt[:-1]).sum() > n // 4  # with ties inside it


def test_introsort_restatement_random(oracle):
    rng = np.random.default_rng(5)
    for n in (0, 1, 16, 17, 300, 4097):
        for k in (2, 7, 1000):
            r = rng.integers(0, k, n).astype(np.float32)
            assert np.array_equal(oracle.std_sort_restated(r)[0], oracle.std_sort_perm(r))
