"""A/B of the SuperPoint forward (BASELINE configs[4] shape: 64 x 640x480 fp16, channels last): the fused
bias + ReLU (+ pool) kernel (fd_nn_bias_relu) and the one-pass first layer (fd_nn_conv3x3_c1) against
the fused path with the matrix-core convolution for 64 -> 64 layers only (FD_SP_C64_ONLY64=1: conv3a,
64 -> 128, on the library), without the matrix-core convolutions (FD_SP_NO_C64=1), without both
(FD_SP_NO_CONV1=1 FD_SP_NO_C64=1: round-3's path) and PyTorch's separate elementwise passes
(FD_SP_UNFUSED=1), interleaved
in one process; prints ms per 64-frame forward. (Sets FD_DEBUG_AB=1: the switches are read only then.)"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from feature_detector_amd import superpoint as sp  # noqa: E402

os.environ["FD_DEBUG_AB"] = "1"
fd.load()
det = sp.NNFeaturePointDetector(sp.Options(kMaxImageRows=480, kMaxImageCols=640))
det.Initialize()
g = torch.Generator(device="cuda")
g.manual_seed(1)
frames = torch.randint(0, 256, (64, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)


def timed(reps=10):
    det.InferenceSession(frames)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        det.InferenceSession(frames)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


MODES = os.environ.get("FD_AB_MODES", "fused,c64_only64,no_c64,no_conv1,unfused").split(",")  # (subset: A/B of builds)
for rnd in range(2):
    for mode in MODES:
        for k in ("FD_SP_UNFUSED", "FD_SP_NO_CONV1", "FD_SP_NO_C64", "FD_SP_C64_ONLY64"):
            os.environ.pop(k, None)
        if mode == "c64_only64":
            os.environ["FD_SP_C64_ONLY64"] = "1"
        if mode == "unfused":
            os.environ["FD_SP_UNFUSED"] = "1"
        elif mode == "no_conv1":
            os.environ["FD_SP_NO_CONV1"] = "1"
            os.environ["FD_SP_NO_C64"] = "1"
        elif mode == "no_c64":
            os.environ["FD_SP_NO_C64"] = "1"
        print(f"round {rnd} {mode}: {timed():.3f} ms per 64-frame forward", flush=True)

