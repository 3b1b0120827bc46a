"""GPU: the pipelined ingest (fd_ingest_*) returns exactly what fd_points_detect
returns for the same frames, across slots reused round-robin with several submits in flight."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}
KIND = {"harris": 0, "shi_tomasi": 1, "fast": 2}


@pytest.mark.parametrize("name", ["harris", "shi_tomasi", "fast"])
def test_ingest_matches_oracle(oracle, name):
    import feature_detector_amd as fd

    rows, cols, batch, depth = 240, 320, 3, 3
    ing = fd.Ingest(name, rows, cols, batch=batch, depth=depth, need=150, min_feature_distance=9)
    frames = [np.stack([oracle.make_frame("noise" if (k + b) % 2 else "checker", 900 + 7 * k + b, rows, cols)
                        for b in range(batch)]) for k in range(7)]
    got = {}
    for k in range(len(frames)):
        slot = k % depth
        if k >= depth:
            got[k - depth] = ing.wait(slot)
        ing.frames(slot)[:] = frames[k]
        ing.submit(slot)
    for k in range(len(frames) - depth, len(frames)):
        got[k] = ing.wait(k % depth)
    for k, fr in enumerate(frames):
        for b in range(batch):
            exp = oracle.detect(KIND[name], fr[b], 9, THR[name], 150, sort_mode=1)[0]
            np.testing.assert_array_equal(got[k][b], exp)
    ing.close()


def test_ingest_misuse():
    import feature_detector_amd as fd

    ing = fd.Ingest("harris", 64, 64, batch=1, depth=2)
    with pytest.raises(fd.FdError):
        ing.wait(0)  # nothing submitted
    ing.frames(0)[:] = 7
    ing.submit(0)
    with pytest.raises(fd.FdError):
        ing.submit(0)  # still pending
    assert [len(x) for x in ing.wait(0)] == [0]  # flat frame: no candidates
    ing.close()
