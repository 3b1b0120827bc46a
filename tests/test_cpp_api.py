"""The C++ drop-in API (include/feature_detector/*, libfeature_detector.so) driven by headless
restatements of the reference demos (tests/cpp/*.cpp mirror test/test_feature_point_detector.cpp and
test/test_feature_line_detector.cpp). GPU tests compare with the oracle / the reference's counts."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "feature_detector_amd", "lib")
KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2, "harris_prior": 0}
THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0, "harris_prior": 30.0}


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "feature_detector_amd", "api")])


def _run(prog, img, tmp_path, *extra):
    raw = tmp_path / "frame.u8"
    np.ascontiguousarray(img, np.uint8).tofile(raw)
    out = subprocess.run([os.path.join(LIB, prog), str(raw), str(img.shape[0]), str(img.shape[1]), *map(str, extra)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    return [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]


def test_api_builds_and_links():
    _build()
    for f in ("libfeature_detector.so", "fd_demo_points", "fd_demo_lines", "fd_demo_descriptor"):
        assert os.path.exists(os.path.join(LIB, f))
    nm = subprocess.run(["nm", "-DC", os.path.join(LIB, "libfeature_detector.so")], capture_output=True, text=True).stdout
    for sym in ("feature_detector::FeaturePointDetector::DetectGoodFeatures",
                "feature_detector::FeaturePointDetector::SparsifyFeatures",
                "feature_detector::FeatureLineDetector::DetectGoodFeatures",
                "feature_detector::BriefDescriptor::ComputeForAllFeatures"):
        assert sym in nm


def test_without_gpu_calls_fail_loudly(tmp_path, image_png):
    """No CPU fallback: without a visible GPU every detector call returns false."""
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    _build()
    res = _run("fd_demo_points", image_png, tmp_path)
    assert all(r["ok"] is False for r in res)


@pytest.mark.gpu
def test_point_demo_matches_oracle(tmp_path, image_png, oracle, ref_counts):
    _build()
    res = {r["test"]: r for r in _run("fd_demo_points", image_png, tmp_path)}
    assert res["null_image"]["ok"] is False
    prior = np.array([(i * 15, j * 15) for i in range(1, 10) for j in range(1, 10)], np.float32)
    for name in ("fast", "harris", "shi_tomasi", "harris_prior"):
        r = res[name]
        assert r["ok"] is True
        feats, cands = oracle.detect(KIND[name], image_png, 20, THR[name], 200,
                                     prior if name == "harris_prior" else None, sort_mode=0)
        assert np.array_equal(np.array(r["features"], np.float32).reshape(-1, 2), feats), name
        assert r["n_candidates"] == len(cands[0])
        if name in ref_counts["image_png"]:
            assert r["n_candidates"] == ref_counts["image_png"][name]["candidates"]
            assert len(r["features"]) == ref_counts["image_png"][name]["features"]
        # candidates() holds the reference's std::sort order (oracle sort_mode 0)
        top = np.array(r["top_candidates"], np.float64)
        n = len(top)
        assert np.array_equal(top[:, 0].astype(np.float32), cands[0][:n])
        assert np.array_equal(top[:, 1].astype(np.int32), cands[1][:n])
        assert np.array_equal(top[:, 2].astype(np.int32), cands[2][:n])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["harris", "shi_tomasi"])
def test_point_demo_tie_frame_reference_order(tmp_path, oracle, name):
    """Equal responses in the greedy scan: the drop-in class runs FD_TIES_REFERENCE, so its features
    are the reference's std::sort order (oracle sort_mode 0), which differs from raster order here."""
    from conftest import make_tie_frame

    img = make_tie_frame(oracle)
    _build()
    r = {x["test"]: x for x in _run("fd_demo_points", img, tmp_path)}[name]
    feats, _ = oracle.detect(KIND[name], img, 20, THR[name], 200, None, sort_mode=0)
    stable, _ = oracle.detect(KIND[name], img, 20, THR[name], 200, None, sort_mode=1)
    got = np.array(r["features"], np.float32).reshape(-1, 2)
    assert np.array_equal(got, feats) and not np.array_equal(got, stable)


@pytest.mark.gpu
def test_line_demo_reference_counts(tmp_path, image_png, oracle, ref_counts):
    _build()
    (r,) = _run("fd_demo_lines", image_png, tmp_path)
    assert r["ok"] is True
    assert r["n_valid"] == ref_counts["image_png"]["lsd_valid"] == r["n_sorted"]
    assert len(r["lines"]) == ref_counts["image_png"]["lsd_lines"]
    assert r["map_passes"] == 1  # pixels() / sorted_pixels() materialised once, on first access
    # members never read: DetectGoodFeatures is the single fd_lsd_lines pass, same segments
    (q,) = _run("fd_demo_lines", image_png, tmp_path, 1)
    assert q["ok"] is True and q["map_passes"] == 0 and q["lines"] == r["lines"]


@pytest.mark.gpu
@pytest.mark.parametrize("rec_i", [0, 1])
def test_line_demo_synthetic_counts(tmp_path, oracle, ref_counts, rec_i):
    rec = ref_counts["synthetic_lsd_lines"][rec_i]
    img = oracle.make_frame(rec["pattern"], 1234, rec["rows"], rec["cols"], rec["period"])
    _build()
    (r,) = _run("fd_demo_lines", img, tmp_path)
    assert len(r["lines"]) == rec["lines"]


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", [0, 1])
def test_descriptor_demo_matches_oracle(tmp_path, image_png, oracle, sampler):
    """test_feature_descriptor.cpp: Harris (dist 20, thr 20, need 10) then BRIEF kLength 128, half 8."""
    _build()
    res = {r["test"]: r for r in _run("fd_demo_descriptor", image_png, tmp_path, sampler)}
    h, b = res["harris"], res["brief"]
    assert h["ok"] is True and b["ok"] is True and b["float_overload_ok"] is True
    feats, _ = oracle.detect(0, image_png, 20, 20.0, 10, None, sort_mode=0)
    xy = np.array(h["features"], np.float32).reshape(-1, 2)
    assert np.array_equal(xy, feats)
    bits, _, _ = oracle.brief(image_png, xy, 128, 8, sampler)
    exp = ["".join(str((w[j >> 5] >> (j & 31)) & 1) for j in range(128)) for w in bits]
    assert b["descriptors"] == exp
    assert res["brief_false_cases"] == {"test": "brief_false_cases", "empty_uv": False, "null_image": False}


@pytest.mark.gpu
@pytest.mark.parametrize("order,dist,prior,base", [("raster", 20, 0, "plain"), ("reverse", 20, 1, "plain"),
                                                    ("twice", 0, 0, "plain"), ("reverse", 1, 0, "plain"),
                                                    ("raster", 20, 0, "harris"), ("reverse", 20, 1, "harris")])
def test_custom_subclass_candidates(tmp_path, image_png, oracle, order, dist, prior, base):
    """A subclass with its own ComputeCandidates (tests/cpp/test_custom_detector.cpp), deriving from
    FeaturePointDetector or from FeaturePointHarrisDetector (overriding only ComputeCandidates, the NVI
    extension point of feature_point_harris_detector.h:24): DetectGoodFeatures calls the override once
    and selects its candidates on the GPU in the reference's order; candidates() and mask() afterwards
    hold what the reference leaves there."""
    from test_gpu_select_custom import PRIOR, gradient_candidates

    _build()
    r = _run("fd_demo_custom", image_png, tmp_path, order, dist, 300, prior, base)[0]
    assert r["ok"] is True and r["calls"] == 1
    rr, xx, yy = gradient_candidates(image_png, order=order)
    pr = PRIOR if prior else None
    feats, (sr, sx, sy) = oracle.select(rr, xx, yy, 480, 752, dist, 300, pr, sort_mode=0, sorted_out=True)
    assert np.array_equal(np.array(r["features"], np.float32).reshape(-1, 2), feats)
    assert r["n_candidates"] == len(rr)
    top = np.array(r["top_candidates"], np.float64)
    assert np.array_equal(top[:, 0].astype(np.float32), sr[:64])
    assert np.array_equal(top[:, 1].astype(np.int32), sx[:64]) and np.array_equal(top[:, 2].astype(np.int32), sy[:64])
    # mask_: prior boxes, then a box per new feature except the one that reached `need` (:67-70)
    m = np.ones((480, 752), bool)
    boxes = (list(PRIOR) if prior else []) + list(feats[:-1] if len(feats) + (81 if prior else 0) >= 300 else feats)
    for fx, fy in boxes:
        r0, c0 = int(fy), int(fx)
        m[max(r0 - dist, 0):max(r0 + dist + 1, 0), max(c0 - dist, 0):max(c0 + dist + 1, 0)] = False
    assert r["mask_zeros"] == int((~m).sum())
