"""CPU: the LSD line oracle (oracle/fd_oracle_lines.cpp, FeatureLineDetector::DetectGoodFeatures in the
reference's data structures) reproduces the reference's recorded line counts and the contract of its
outputs. The counts come from the survey's probe (stand-in headers: a consistency check, not a pin;
DESIGN.md §3); the CircularBuffer overflow policy and AngleDiffInRad are unpinned assumptions."""
import numpy as np
import pytest


def test_image_png_lines(oracle, image_png):
    lines = oracle.lsd_lines(image_png)
    assert len(lines) == 40  # 40 lines


@pytest.mark.parametrize("rows,cols,expect", [(480, 640, 112), (1080, 1920, 792)])
def test_checker64_lines(oracle, ref_counts, rows, cols, expect):
    rec = [r for r in ref_counts["synthetic_lsd_lines"] if r["rows"] == rows][0]
    assert rec["lines"] == expect
    img = oracle.make_frame("checker", 1234, rows, cols, 64)
    assert len(oracle.lsd_lines(img)) == expect


def test_line_contract(oracle, image_png):
    lines = oracle.lsd_lines(image_png)
    R, C = image_png.shape
    assert (lines[:, 6] >= 20.0).all()  # length >= kMinValidLineLengthInPixel (:40)
    assert (lines[:, 11] >= 0.6).all()  # inlier ratio >= kMaxToleranceInlierRation (:40)
    xs, ys = lines[:, [0, 2]], lines[:, [1, 3]]
    assert (xs > -2).all() and (xs < C + 2).all() and (ys > -2).all() and (ys < R + 2).all()
    d = np.hypot(lines[:, 9], lines[:, 10])
    assert np.allclose(d, 1.0, atol=1e-6)  # unit direction (cos, sin)


def test_needed_zero_and_tiny_frames(oracle, image_png):
    assert len(oracle.lsd_lines(image_png, needed=0)) == 0  # :15
    for shape in ((2, 2), (3, 3), (4, 5), (5, 4)):
        assert len(oracle.lsd_lines(np.zeros(shape, np.uint8))) == 0


def test_ramp_overflows_ring_but_is_deterministic(oracle):
    # a smooth diagonal ramp: one huge aligned region whose BFS frontier exceeds the 1000-entry
    # CircularBuffer (overflow policy assumed: drop the oldest); the result must at least be stable
    r, c = np.mgrid[0:400, 0:600]
    img = ((r * 3 + c * 5) % 256).astype(np.uint8)
    a, b = oracle.lsd_lines(img), oracle.lsd_lines(img)
    assert np.array_equal(a, b)
