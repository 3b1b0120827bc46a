"""Diagnostic: wall time of SuperPoint Initialize (MIOpen solver choice) + network time, under the
MIOpen env the caller sets (tools/gpu_sp_find_probe.sh)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from feature_detector_amd import superpoint as spm  # noqa: E402

t0 = time.time()
det = spm.SuperPointDetector(spm.Options(kComputeDescriptors=True, kMaxImageRows=480, kMaxImageCols=640))
det.Initialize()
frames = torch.randint(0, 256, (64, 480, 640), device="cuda", dtype=torch.int32).to(torch.uint8)
det.InferenceSession(frames)
torch.cuda.synchronize()
t1 = time.time()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(5):
    det.InferenceSession(frames)
e.record()
torch.cuda.synchronize()
print("%s init+first %.1f s, network %.2f ms / 64 frames" % (os.environ.get("PROBE", ""), t1 - t0, s.elapsed_time(e) / 5))
