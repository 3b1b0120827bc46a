"""Kernel-level profile driver (run under rocprofv3 --kernel-trace --stats): the SuperPoint forward on 64
640x480 frames, 5 calls, in the current configuration (FD_SP_* switches apply)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from feature_detector_amd import superpoint as sp  # noqa: E402

fd.load()
det = sp.NNFeaturePointDetector(sp.Options(kMaxImageRows=480, kMaxImageCols=640))
det.Initialize()
g = torch.Generator(device="cuda")
g.manual_seed(1)
frames = torch.randint(0, 256, (64, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
for _ in range(5):
    det.InferenceSession(frames)
torch.cuda.synchronize()
print("done")
