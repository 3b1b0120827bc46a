"""k_select_reference phase clocks on the bench's own tie frames (run with FD_SELECT_STAMPS=1: the
library prints the clocks of every re-selected frame to stderr): the headline pool (640x480 Harris,
batch 1 x 16 seeds) and one north-star batch (1920x1080 Shi-Tomasi x256)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("FD_DEBUG_AB", "1")
os.environ.setdefault("FD_SELECT_STAMPS", "1")
import torch  # noqa: E402

import bench  # noqa: E402
import feature_detector_amd as fd  # noqa: E402

dev = torch.device("cuda", 0)
for i in range(16):
    f = bench.make_frames(torch, "noise", 1, 480, 640, 1234 + 7919 * i, dev)
    fd.detect_points("harris", f, 200, 20, 30.0, ties="reference")
    torch.cuda.synchronize()
if "--headline-only" not in sys.argv:
    f = bench.make_frames(torch, "noise", 256, 1080, 1920, 99, dev)
    fd.detect_points("shi_tomasi", f, 200, 20, 40.0, ties="reference")
    torch.cuda.synchronize()
print("done")
