"""Timing-only diagnostic for knockout builds (FD_LIB_PATH=...): 200 headline detect calls (Harris
640x480 batch 1), exceptions from the selection's consistency guards swallowed (a knockout build may
feed it inconsistent input); run under rocprofv3 --kernel-trace --stats for the per-kernel durations."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

g = torch.Generator(device="cuda")
g.manual_seed(7)
fr = torch.randint(0, 256, (1, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
errs = 0
for _ in range(200):
    try:
        fd.detect_points("harris", fr, 200, 20, 30.0, ties="raster")
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 -- diagnostic: a knockout build trips the selection's guards
        errs += 1
print("calls 200, guard errors", errs)
