"""K10 (fd_nn_conv3x3_c64) alone at one SuperPoint layer's shape (64 frames of 640x480 input), for
rocprofv3 kernel-trace / PMC passes and quick timing: random fp16 channels-last input and filter, `--calls`
calls after one warm-up call; prints the event-timed average per call and the layer's MFMA floor.
usage: python3 tools/sp_k10_probe.py [--layer conv1b|conv2a|conv2b|conv3a] [--calls N]"""
import argparse
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from feature_detector_amd import superpoint as sp  # noqa: E402

LAYERS = {"conv1b": (480, 640, 64, True, 64), "conv2a": (240, 320, 64, False, 64), "conv2b": (240, 320, 64, True, 64),
          "conv3a": (120, 160, 128, False, 64)}
ap = argparse.ArgumentParser()
ap.add_argument("--layer", default="conv1b", choices=sorted(LAYERS))
ap.add_argument("--calls", type=int, default=5)
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--zero", action="store_true", help="all-zero input (the matrix cores' power draw on zeros vs random)")
a = ap.parse_args()
h, w, co, pool, cin = LAYERS[a.layer]
fd.load()
g = torch.Generator(device="cuda")
g.manual_seed(7)
x = (torch.rand((a.frames, cin, h, w), generator=g, device="cuda") * 2).half().contiguous(memory_format=torch.channels_last)
if a.zero:
    x.zero_()
wt = (torch.randn((co, cin, 3, 3), generator=g, device="cuda") * 0.05).half()
b = (torch.randn((co,), generator=g, device="cuda") * 0.1).half()
packed = [sp.pack_conv3x3_weight(wt[k:k + 64]) for k in range(0, co, 64)]
conv = sp.conv64_bias_relu
out = conv(x, wt, b, pool=pool, packed=packed)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.calls):
    conv(x, wt, b, pool=pool, out=out, packed=packed)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.calls
flop = 2.0 * a.frames * h * w * co * cin * 9
print(f"{a.layer}{' (zero input)' if a.zero else ''}: {ms * 1e3:.1f} us per call, {flop / ms / 1e9:.1f} TFLOP/s "
      f"(MFMA floor at 2.4 GHz {flop / 2.5e15 * 1e6:.0f} us)", flush=True)
