import json
import os
import sys
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


def _read_png_gray(path):
    """Minimal PNG decoder for 8-bit grayscale, non-interlaced (no PIL dependency)."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    w = h = None
    while pos < len(data):
        n = int.from_bytes(data[pos:pos + 4], "big")
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            w, h = int.from_bytes(body[0:4], "big"), int.from_bytes(body[4:8], "big")
            depth, ctype, interlace = body[8], body[9], body[12]
            assert depth == 8 and ctype == 0 and interlace == 0, "only 8-bit gray PNG supported"
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    out = np.zeros((h, w), np.uint8)
    prev = np.zeros(w, np.int32)
    stride = w + 1
    for r in range(h):
        ft = raw[r * stride]
        line = np.frombuffer(raw, np.uint8, w, r * stride + 1).astype(np.int32)
        cur = np.zeros(w, np.int32)
        if ft == 0:
            cur = line
        elif ft == 2:
            cur = (line + prev) & 0xFF
        else:
            for c in range(w):
                a = cur[c - 1] if c > 0 else 0
                b = prev[c]
                cc = prev[c - 1] if c > 0 else 0
                if ft == 1:
                    p = a
                elif ft == 3:
                    p = (a + b) // 2
                else:  # Paeth
                    pa, pb, pc = abs(b - cc), abs(a - cc), abs(a + b - 2 * cc)
                    p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else cc)
                cur[c] = (line[c] + p) & 0xFF
        out[r] = cur
        prev = cur
    return out


@pytest.fixture(scope="session")
def image_png():
    return _read_png_gray(os.path.join(GOLDEN, "image.png"))


@pytest.fixture(scope="session")
def ref_counts():
    with open(os.path.join(GOLDEN, "reference_counts.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.lib()
    return O


def make_tie_frame(oracle, rows=480, cols=640, seed=77, copies=(6, 8)):
    """A frame whose greedy scan meets equal responses: identical 15x15 corner stamps (constant
    surround, so every copy has bit-identical Harris / Shi-Tomasi responses) on a low-contrast noise
    background. The reference's unstable std::sort orders the equal responses differently from raster
    order, so the two tie orders select different feature lists (checked against the oracle)."""
    img = oracle.make_frame("noise", seed, rows, cols) // 4
    patch = np.full((15, 15), 100, np.uint8)
    patch[4:8, 4:8] = 250
    patch[7:11, 7:11] = 10
    ys = np.linspace(10, rows - 30, copies[0]).astype(int)
    xs = np.linspace(10, cols - 30, copies[1]).astype(int)
    for y in ys:
        for x in xs:
            img[y:y + 15, x:x + 15] = patch
    return img
