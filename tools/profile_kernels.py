"""Profiling driver (run under rocprofv3): the bench shapes' kernels only, a fixed number of times.

  --shape bench      fd_points_detect, Harris, 640x480, batch 1 (BASELINE configs[1]), 200 calls
  --shape northstar  fd_points_response (per-pixel kernel alone), Shi-Tomasi 1920x1080 batch 256, 10 calls
"""
import argparse
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--shape", default="bench", choices=["bench", "northstar", "fast720"])
p.add_argument("--calls", type=int, default=0)
a = p.parse_args()
g = torch.Generator(device="cuda")
g.manual_seed(7)
if a.shape == "bench":
    frames = torch.randint(0, 256, (1, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
    for _ in range(a.calls or 200):
        fd.detect_points("harris", frames, 200, 20, 30.0)
elif a.shape == "northstar":
    frames = torch.randint(0, 256, (256, 1080, 1920), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
    for _ in range(a.calls or 10):
        fd.point_response("shi_tomasi", frames, 40.0)
else:
    frames = torch.randint(0, 256, (64, 720, 1280), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
    for _ in range(a.calls or 10):
        fd.detect_points("fast", frames, 200, 20, 10.0)
torch.cuda.synchronize()
print("done", a.shape)
