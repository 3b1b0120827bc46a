"""Diagnostic: k_select phase clocks (FD_SELECT_STAMPS=1) at BASELINE configs[2] (FAST 1280x720 x64 noise)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for kv in sys.argv[1:]:  # VAR=VALUE settings for the library (A/B switches), before it is loaded
    k, v = kv.split("=", 1)
    os.environ[k] = v
os.environ.setdefault("FD_DEBUG_AB", "1")
os.environ.setdefault("FD_SELECT_STAMPS", "1")
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

g = torch.Generator(device="cuda")
g.manual_seed(7)
frames = torch.randint(0, 256, (64, 720, 1280), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
for _ in range(3):
    fd.detect_points("fast", frames, 200, 20, 10.0, ties="raster")
    torch.cuda.synchronize()
