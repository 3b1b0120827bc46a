"""CPU: the oracle's SuperPoint post-processing against a second, pure-Python
restatement of nn_feature_point_detector.cpp:59-73 (CreateMask), :128-155 (multimap candidates +
greedy box selection) and :163-193 (bilinear descriptor sampling), including the std::multimap tie
order (equal responses are walked in descending raster order from crbegin)."""
import math

import numpy as np
import pytest

F = np.float32


def py_nn_select(heat, border, dist, max_features, thr, prior):
    R, C = heat.shape
    mask = np.ones((R, C), bool)
    if border:
        mask[:border] = False
        mask[R - border:] = False
        mask[:, :border] = False
        mask[:, C - border:] = False

    def draw(r, c):
        mask[max(0, r - dist):min(R - 1, r + dist) + 1, max(0, c - dist):min(C - 1, c + dist) + 1] = False

    for x, y in prior:
        draw(int(F(y)), int(F(x)))
    cands = [(heat[r, c], r * C + c) for r in range(R) for c in range(C) if heat[r, c] > F(thr)]
    cands.sort(key=lambda t: (-t[0], -t[1]))  # multimap walked from crbegin
    out, size = [], len(prior)
    for _, i in cands:
        r, c = divmod(i, C)
        if not mask[r, c]:
            continue
        out.append((c, r))
        size += 1
        if size >= max_features:
            break
        draw(r, c)
    return np.array(out, np.float32).reshape(-1, 2)


@pytest.mark.parametrize("border,dist,maxf,thr", [(3, 15, 240, 0.1), (0, 4, 30, 0.5), (5, 0, 50, 0.3), (3, 15, 1, 0.1)])
def test_nn_select_matches_python(oracle, border, dist, maxf, thr):
    rng = np.random.default_rng(border * 100 + dist)
    heat = (np.round(rng.random((48, 64)) * 16) / 16).astype(np.float32)  # coarse values: many ties
    for prior in ([], [(10.7, 20.2), (50.0, 3.0)]):
        got = oracle.nn_select(heat, border, dist, maxf, thr, prior if prior else None)
        exp = py_nn_select(heat, border, dist, maxf, thr, prior)
        assert np.array_equal(got, exp)


def test_nn_select_tie_order_is_reverse_raster(oracle):
    heat = np.zeros((20, 20), np.float32)
    heat[5, 5] = heat[5, 12] = heat[14, 5] = 0.5  # equal responses, far apart
    got = oracle.nn_select(heat, 0, 2, 10, 0.1)
    assert got.tolist() == [[5, 14], [12, 5], [5, 5]]


def test_nn_descriptors_matches_python(oracle):
    rng = np.random.default_rng(5)
    m = rng.standard_normal((7, 6, 9)).astype(np.float32)
    xy = np.array([(0, 0), (8, 8), (12.5, 20.25), (63.9, 39.9), (64, 40), (-3, 4), (-0.5, 10), (7.99, 7.99)], np.float32)
    got = oracle.nn_descriptors(m, xy)
    for i, (x, y) in enumerate(xy):
        row, col = F(y) / F(8), F(x) / F(8)
        ir, ic = int(row), int(col)
        sr, sc = F(row - F(math.floor(row))), F(col - F(math.floor(col)))
        w = [F(F(1) - sc) * F(F(1) - sr), sc * F(F(1) - sr), F(F(1) - sc) * sr, sc * sr]
        for j in range(7):
            if ir < 0 or ir >= 6 - 1 or ic < 0 or ic >= 9 - 1:
                e = F(0)
            else:
                e = F(F(F(w[0] * m[j, ir, ic]) + F(w[1] * m[j, ir, ic + 1])) + F(w[2] * m[j, ir + 1, ic])) + F(w[3] * m[j, ir + 1, ic + 1])
            assert got[i, j].view(np.uint32) == np.float32(e).view(np.uint32), (i, j)
