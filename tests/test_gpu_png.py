"""GPU: fd_png_frames (host decode threads -> one upload -> colour -> gray on the GPU) equals the host
decoder image by image, feeds detection directly, and the C++ demo's LoadImage path (PNG file in,
as the reference demo at test/test_feature_point_detector.cpp:104) gives the raw-frame results."""
import json
import os
import subprocess

import numpy as np
import pytest

from png_util import encode_png

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("ch", [1, 2, 3, 4])
def test_png_frames_match_host_decode(ch, oracle):
    import torch

    import feature_detector_amd as fd

    rng = np.random.default_rng(10 + ch)
    imgs = []
    for i in range(5):
        base = oracle.make_frame("checker", 50 + i, 97, 131, 16)
        img = np.stack([np.roll(base, k, axis=1) for k in range(ch)], -1) if ch > 1 else base
        imgs.append(img)
    pngs = [encode_png(x, filters=(i % 5, 4, 1, 3, 2, 0)) for i, x in enumerate(imgs)]
    dev = fd.png_frames(pngs, threads=3)
    torch.cuda.synchronize()
    host = np.stack([fd.load_png(p) for p in pngs])
    assert np.array_equal(dev.cpu().numpy(), host)


def test_png_frames_detect(image_png, oracle):
    import torch

    import feature_detector_amd as fd

    data = open(os.path.join(ROOT, "tests", "golden", "image.png"), "rb").read()
    frames = fd.png_frames([data, data])
    res = fd.detect_points("harris", frames, 200, 20, 30.0)
    torch.cuda.synchronize()
    exp, _ = oracle.detect(0, image_png, 20, 30.0, 200, sort_mode=0)
    assert np.array_equal(res.features(0), exp) and np.array_equal(res.features(1), exp)


def test_demo_loads_png(tmp_path, image_png):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "feature_detector_amd", "api")])
    lib = os.path.join(ROOT, "feature_detector_amd", "lib")
    raw = tmp_path / "f.u8"
    image_png.tofile(raw)
    a = subprocess.run([os.path.join(lib, "fd_demo_points"), str(raw), "480", "752"], capture_output=True, text=True,
                       timeout=300)
    b = subprocess.run([os.path.join(lib, "fd_demo_points"), os.path.join(ROOT, "tests", "golden", "image.png")],
                       capture_output=True, text=True, timeout=300)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    ja = [json.loads(x) for x in a.stdout.splitlines() if x.startswith("{")]
    jb = [json.loads(x) for x in b.stdout.splitlines() if x.startswith("{")]
    assert ja == jb and len(ja) >= 4


@pytest.mark.parametrize("ch", [1, 3])
def test_png_frames_out_unaligned_and_checked(ch, oracle):
    """out= may start at any byte (the converter stores dwords only when both ends are 4-byte aligned);
    a wrong shape, dtype or device raises before any work is queued."""
    import torch

    import feature_detector_amd as fd

    imgs = [oracle.make_frame("noise", 70 + i, 33, 50) for i in range(3)]
    if ch == 3:
        imgs = [np.stack([x, np.roll(x, 1, 0), np.roll(x, 2, 1)], -1) for x in imgs]
    pngs = [encode_png(x) for x in imgs]
    host = np.stack([fd.load_png(p) for p in pngs])
    big = torch.full((host.size + 8,), 0xA5, dtype=torch.uint8, device="cuda")
    for off in (1, 2, 3):
        big.fill_(0xA5)
        out = big[off:off + host.size].view(host.shape)
        fd.png_frames(pngs, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), host)
        b = big.cpu().numpy()
        assert (b[:off] == 0xA5).all() and (b[off + host.size:] == 0xA5).all()
    for bad in (torch.empty((3, 33, 49), dtype=torch.uint8, device="cuda"),
                torch.empty((3, 33, 50), dtype=torch.int32, device="cuda"),
                torch.empty((3, 33, 50), dtype=torch.uint8)):
        with pytest.raises(ValueError):
            fd.png_frames(pngs, out=bad)
