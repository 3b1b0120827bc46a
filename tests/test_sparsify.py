"""FeaturePointDetector::SparsifyFeatures (reference feature_point_detector.cpp:27-52) of the C++
drop-in against the oracle's restatement (orc_sparsify). Host-only code: runs without a GPU."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "feature_detector_amd", "lib", "fd_demo_sparsify")


def _run(xy, status, rows, cols, gr, gc, need, after):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "feature_detector_amd", "api")])
    lines = [str(len(xy))] + [f"{x!r} {y!r} {s}" for (x, y), s in zip(xy.tolist(), status)]
    out = subprocess.run([EXE, str(rows), str(cols), str(gr), str(gc), str(need), str(after)],
                         input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout)


@pytest.mark.parametrize("seed", range(6))
def test_sparsify_matches_oracle(oracle, seed):
    rng = np.random.default_rng(seed)
    rows, cols = [(480, 752), (480, 640), (1080, 1920), (100, 37), (12, 12), (479, 641)][seed]
    gr, gc = [(12, 12), (12, 12), (8, 16), (5, 3), (12, 12), (2, 7)][seed]
    n = int(rng.integers(0, 400))
    # features inside, on the border, and outside the image (negative or past the last cell)
    xy = np.stack([rng.uniform(-30, cols + 30, n), rng.uniform(-30, rows + 30, n)], 1).astype(np.float32)
    xy[: n // 4] = np.floor(xy[: n // 4])  # integer pixel positions, as detectors produce
    need, after = (1, 0) if seed % 2 == 0 else (2, 5)
    status = rng.choice([need, after, 3], size=n).astype(np.uint8)
    got = _run(xy, status.tolist(), rows, cols, gr, gc, need, after)
    est, emask = oracle.sparsify(xy, rows, cols, gr, gc, need, after, status.copy())
    assert got["status"] == est.tolist()
    assert got["mask"] == emask.reshape(-1).tolist()


def test_sparsify_resets_mismatched_status(oracle):
    # status of another size is reset to all ones before filtering (:29-31)
    xy = np.array([(10, 10), (12, 11), (400, 300), (401, 300)], np.float32)
    got = _run(xy, [-1] * len(xy), 480, 640, 12, 12, 1, 0)
    est, emask = oracle.sparsify(xy, 480, 640, 12, 12, 1, 0, None)
    assert got["status"] == est.tolist() == [1, 0, 1, 0]
    assert got["mask"] == emask.reshape(-1).tolist()
