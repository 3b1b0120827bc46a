"""A/B (diagnostic): fd_lsd_lines on BASELINE configs[3] (256 frames of 1920x1080 64-px checker + noise,
the bench's frames), seed order on the GPU (default) against the host std::sort (FD_LSD_HOST_SORT=1),
and with the order copied from a device buffer
(FD_LSD_ORD_MAPPED=0) instead of written into pinned host memory, alternating, `reps` timed calls each; the library's phase line (FD_LINES_TIMING) goes to stderr.
usage: python3 tools/lines_ab.py [reps] [batch]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["FD_DEBUG_AB"] = "1"
os.environ["FD_LINES_TIMING"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import feature_detector_amd as fd  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
frames = bench.make_frames(torch, "checker", batch, 1080, 1920, 0, "cuda", period=64)
torch.cuda.synchronize()
ref = None
MODES = os.environ.get("FD_AB_MODES", "gpu,gpu_copy,host").split(",")  # (gpu_narrow: no wide prelude)
for mode in MODES + MODES:
    os.environ["FD_LSD_HOST_SORT"] = "1" if mode == "host" else "0"
    os.environ["FD_LSD_ORD_MAPPED"] = "0" if mode == "gpu_copy" else "1"  # (gpu_copy: ord via a device buffer)
    if mode == "gpu_narrow":
        os.environ["FD_LSD_WIDE"] = "0"
    else:
        os.environ.pop("FD_LSD_WIDE", None)
    segs = fd.lsd_lines(frames, max_lines=2048)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        segs = fd.lsd_lines(frames, max_lines=2048)
    ms = (time.perf_counter() - t0) * 1e3 / reps
    same = None
    if ref is None:
        ref = segs
    else:
        same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(ref, segs))
    print(f"{mode}: {ms:.2f} ms per batch of {batch}, {sum(len(s) for s in segs)} lines, same as first: {same}",
          flush=True)
