"""CPU: the BRIEF pattern table and the oracle's BRIEF restatement.

* The generated GPU pattern table (feature_detector_amd/csrc/fd_brief_pattern.inc) equals the
  reference's pattern_idx_ (descriptor_brief.cpp:52-309), re-parsed from the reference source when it is
  present (this container; the GPU box has no /root/reference).
* The C oracle (oracle/fd_oracle.cpp orc_brief) equals a second, independent restatement written here
  with numpy float32 scalars (IEEE single, no FMA), op for op after descriptor_brief.cpp:8-50, for both
  samplers, integral and fractional keypoints, several lengths and patch sizes.
* Properties the reference fixes whatever its sampler: border keypoints and flat patches give the
  all-zero descriptor (:10, :15-17, :30); at integer keypoints the moments do not depend on the sampler.
The sampled bits themselves are parity-unpinned (the reference's float sampler is un-vendored).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BRIEF = "/root/reference/src/feature_descriptor/descriptor_brief.cpp"
F = np.float32


@pytest.fixture(scope="module")
def orc(oracle):
    return oracle


@pytest.mark.skipif(not os.path.exists(REF_BRIEF), reason="reference source not present")
def test_pattern_table_matches_reference():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_brief_pattern as g

    ref = g.parse_pattern(REF_BRIEF)
    words = g.read_inc()
    assert len(words) == 256
    assert g.unpack(words) == ref


def test_pattern_table_shape(orc):
    pat = orc.brief_pattern()
    assert pat.shape == (1024,)
    assert np.abs(pat).max() <= 13  # "Pattern max offset is 13" (descriptor_brief.cpp:12)


def _pix(img, r, c):
    R, C = img.shape
    i = int(r) * C + int(c)
    return F(img.reshape(-1)[i]) if 0 <= i < R * C else F(0)


def _sample(img, row, col, sampler):
    r0, c0 = int(row), int(col)  # static_cast<int32_t>: truncation toward zero
    if sampler == 1:
        return _pix(img, r0, c0)
    ex = F(col) - F(c0)
    ey = F(row) - F(r0)
    ex1, ey1 = F(1) - ex, F(1) - ey
    return (ex1 * ey1 * _pix(img, r0, c0) + ex * ey1 * _pix(img, r0, c0 + 1) + ex1 * ey * _pix(img, r0 + 1, c0)
            + ex * ey * _pix(img, r0 + 1, c0 + 1))


def numpy_brief(img, x, y, length, half, sampler, pat):
    """descriptor_brief.cpp:8-50 with numpy float32 scalars."""
    R, C = img.shape
    x, y = F(x), F(y)
    nw = (length + 31) // 32
    bits = np.zeros(nw, np.uint32)
    mb = max(F(19.0), F(half) * F(2.0))
    if x < mb or x > F(C) - mb or y < mb or y > F(R) - mb:
        return bits, 0, None
    m01, m10 = F(0), F(0)
    for dx in range(-half, half + 1):
        for dy in range(-half, half + 1):
            v = _sample(img, y + F(dy), x + F(dx), sampler)
            m10 = F(m10 + F(dx) * v)
            m01 = F(m01 + F(dy) * v)
    m = np.sqrt(F(m01 * m01 + m10 * m10), dtype=F)
    if m < F(1e-6):
        return bits, 0, (m10, m01, m)
    s, c = F(m01 / m), F(m10 / m)
    for i in range(length):
        ax, ay, bx, by = (F(v) for v in pat[4 * i:4 * i + 4])
        p1x, p1y = F(F(c * ax) + F(-s * ay)) + x, F(F(s * ax) + F(c * ay)) + y
        p2x, p2y = F(F(c * bx) + F(-s * by)) + x, F(F(s * bx) + F(c * by)) + y
        if _sample(img, p1y, p1x, sampler) < _sample(img, p2y, p2x, sampler):
            bits[i >> 5] |= np.uint32(1 << (i & 31))
    return bits, 1, (m10, m01, m)


@pytest.mark.parametrize("sampler", [0, 1])
@pytest.mark.parametrize("length,half", [(256, 8), (128, 8), (33, 3), (1, 0), (64, 12)])
def test_oracle_matches_numpy_restatement(orc, sampler, length, half):
    img = orc.make_frame("noise", 77 + length, 96, 112)
    rng = np.random.default_rng(length * 7 + half)
    pts = [(40.0, 40.0), (56.0, 47.0), (30.25, 60.5), (70.75, 33.125), (20.0, 20.0), (10.0, 50.0), (90.0, 76.9)]
    pts += [(float(rng.uniform(25, 85)), float(rng.uniform(25, 70))) for _ in range(3)]
    uv = np.array(pts, np.float32)
    bits, valid, mom = orc.brief(img, uv, length, half, sampler)
    pat = orc.brief_pattern()
    for k, (x, y) in enumerate(uv):
        eb, ev, em = numpy_brief(img, x, y, length, half, sampler, pat)
        assert valid[k] == ev, k
        assert np.array_equal(bits[k], eb), k
        if em is not None:
            assert np.array_equal(mom[k].view(np.uint32), np.array(em, np.float32).view(np.uint32)), k


def test_border_flat_and_sampler_independent_moments(orc):
    img = orc.make_frame("checker", 5, 120, 160)
    uv = np.array([(18.9, 60), (19, 60), (141, 60), (141.5, 60), (80, 18), (80, 101), (80, 101.5), (80, 60)],
                  np.float32)
    b0, v0, m0 = orc.brief(img, uv, 256, 8, 0)
    b1, v1, m1 = orc.brief(img, uv, 256, 8, 1)
    assert v0.tolist() == [0, 1, 1, 0, 0, 1, 0, 1] == v1.tolist()
    assert not b0[v0 == 0].any() and not b1[v1 == 0].any()
    # integer keypoints: both samplers read the pixel itself, so moments and orientation agree
    assert np.array_equal(m0[v0 == 1], m1[v1 == 1])
    flat = np.full((64, 64), 77, np.uint8)
    bf, vf, mf = orc.brief(flat, np.array([(32, 32)], np.float32), 256, 8, 0)
    assert vf[0] == 0 and not bf.any() and mf[0, 2] == 0  # m == 0 -> RETURN_FALSE_IF (:30)
    # kHalfPatchSize 12 raises the border to 24 (:14)
    _, v12, _ = orc.brief(img, np.array([(23.5, 60), (24, 60)], np.float32), 256, 12, 0)
    assert v12.tolist() == [0, 1]
