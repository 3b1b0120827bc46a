"""CPU: the PNG front end (fd_png_info / fd_png_decode) against a numpy reference
decoder on encoder-made images (every row filter, every supported colour type), the reference's
examples/image.png fixture and, when the reference tree is present, its examples/image2.png (RGB).
The colour -> gray conversion of the reference's Visualizor2D::LoadImage is un-vendored: the library's
BT.601 fixed-point rule is checked for self-consistency only (parity unpinned)."""
import os

import numpy as np
import pytest

from png_util import decode_png, encode_png, gray_of


@pytest.mark.parametrize("ch", [1, 2, 3, 4])
def test_roundtrip_all_filters(ch):
    import feature_detector_amd as fd

    rng = np.random.default_rng(ch)
    img = rng.integers(0, 256, (37, 53, ch) if ch > 1 else (37, 53)).astype(np.uint8)
    data = encode_png(img)
    assert fd.png_info(data) == (37, 53, ch)
    got = fd.load_png(data)
    exp = gray_of(img if img.ndim == 3 else img[:, :, None])
    assert np.array_equal(got, exp)


def test_image_png_fixture(image_png):
    import feature_detector_amd as fd

    got = fd.load_png(os.path.join(os.path.dirname(__file__), "golden", "image.png"))
    assert np.array_equal(got, image_png)


@pytest.mark.skipif(not os.path.exists("/root/reference/examples/image2.png"), reason="reference tree absent")
def test_reference_image2_rgb():
    import feature_detector_amd as fd

    data = open("/root/reference/examples/image2.png", "rb").read()
    assert fd.png_info(data) == (480, 640, 3)
    got = fd.load_png(data)
    assert np.array_equal(got, gray_of(decode_png(data)))


def test_rejects_bad_input():
    import feature_detector_amd as fd

    data = encode_png(np.zeros((8, 8), np.uint8))
    with pytest.raises(fd.FdError):
        fd.load_png(data[:40])  # truncated
    with pytest.raises(fd.FdError):
        fd.load_png(b"not a png at all, not even close")
    bad = bytearray(data)
    bad[8 + 8 + 8] = 16  # IHDR bit depth 16
    with pytest.raises(fd.FdError):
        fd.load_png(bytes(bad))
