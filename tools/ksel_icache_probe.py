"""The headline selection (Harris 640x480 batch 1, raster tie order, device outputs) called 200 times,
for rocprofv3 --pmc passes on k_select (instruction-cache counters; tools/ksel_icache.sh)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

g = torch.Generator(device="cuda")
g.manual_seed(7)
fr = torch.randint(0, 256, (16, 1, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
out = (torch.empty((1, 201, 2), dtype=torch.float32, device="cuda"), torch.empty((1,), dtype=torch.int32, device="cuda"),
       torch.empty((1,), dtype=torch.int32, device="cuda"))
for i in range(200):
    fd.detect_points("harris", fr[i % 16], 200, 20, 30.0, out=out, ties="raster")
torch.cuda.synchronize()
print("done")
