"""K1 at the bench shape (Harris 640x480, batch 1): detect (list + level-0 histogram) vs response
(list only) under different tile geometries; run under rocprofv3 --kernel-trace."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

g = torch.Generator(device="cuda")
g.manual_seed(7)
fr = torch.randint(0, 256, (1, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
out = (torch.empty((1, 480 * 640 // 2 + 64), dtype=torch.float32, device="cuda"),
       torch.empty((1, 480 * 640 // 2 + 64), dtype=torch.int32, device="cuda"), torch.empty((1,), dtype=torch.int32, device="cuda"))
mode = sys.argv[1]
for _ in range(100):
    if mode == "detect":
        fd.detect_points("harris", fr, 200, 20, 30.0)
    else:
        fd.point_response("harris", fr, 30.0, out=out)
torch.cuda.synchronize()
