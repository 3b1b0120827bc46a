"""CPU: the reference-data-flow restatement (oracle/fd_oracle_refflow.cpp: float sliding sums, dense
response map, pair list, std::sort, int32 mask -- the timed CPU baseline) selects exactly the features
of the integer-tensor oracle in its reference std::sort mode (sort_mode=0)."""
import numpy as np
import pytest

KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2}
THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}


@pytest.mark.parametrize("name", list(KIND))
def test_refflow_matches_oracle_image_png(oracle, image_png, name):
    det = oracle.RefFlowDetector()
    got = det.detect(KIND[name], image_png, 20, THR[name], 200)
    exp, _ = oracle.detect(KIND[name], image_png, 20, THR[name], 200, sort_mode=0)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("pattern", ["noise", "checker"])
@pytest.mark.parametrize("name", list(KIND))
def test_refflow_matches_oracle_synthetic(oracle, pattern, name):
    det = oracle.RefFlowDetector()
    for seed, (rows, cols) in ((1234, (480, 640)), (77, (131, 203))):
        img = oracle.make_frame(pattern, seed, rows, cols)
        for need, dist in ((200, 20), (1000, 3)):
            got = det.detect(KIND[name], img, dist, THR[name], need)
            exp, _ = oracle.detect(KIND[name], img, dist, THR[name], need, sort_mode=0)
            assert np.array_equal(got, exp), (seed, need, dist)
