"""K9 (fd_nn_conv3x3_c1, SuperPoint conv1a) alone on 64 640x480 fp16 frames: event-timed average of 10
calls after a warm-up call (the library from FD_LIB_PATH when set)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from feature_detector_amd import superpoint as sp  # noqa: E402

fd.load()
g = torch.Generator(device="cuda")
g.manual_seed(3)
x = torch.rand((64, 1, 480, 640), generator=g, device="cuda").half()
wt = (torch.randn((64, 1, 3, 3), generator=g, device="cuda") * 0.5).half()
b = (torch.randn((64,), generator=g, device="cuda") * 0.1).half()
out = sp.conv1_bias_relu(x, wt, b)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    sp.conv1_bias_relu(x, wt, b, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
tag = os.path.basename(os.environ.get("FD_LIB_PATH", "") or "libfdhip.so")
print(f"{tag} conv1a: {ms * 1e3:.1f} us per call, {out.numel() * 2 / ms / 1e9:.0f} GB/s of writes", flush=True)
