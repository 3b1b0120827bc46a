"""The SuperPoint forward on SP_BATCH (default 64) 640x480 frames (BASELINE configs[4] shape), event-timed: prints ms per
64-frame forward for two rounds of 10 calls (the library from FD_LIB_PATH when set)."""
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
NB = int(os.environ.get("SP_BATCH", "64"))  # frames per network batch
frames = torch.randint(0, 256, (NB, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
for _ in range(3):
    det.InferenceSession(frames)
torch.cuda.synchronize()
tag = os.path.basename(os.environ.get("FD_LIB_PATH", "") or "libfdhip.so")
for rnd in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        det.InferenceSession(frames)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{tag} round {rnd}: {ms:.3f} ms per {NB}-frame forward ({ms * 64 / NB:.3f} ms per 64 frames)", flush=True)
