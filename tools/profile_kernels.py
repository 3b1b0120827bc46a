"""Profiling driver (run under rocprofv3 --kernel-trace --stats): the bench shapes' kernels only, a
fixed number of times, on seeded uniform-noise frames generated on the GPU.

  --shape bench      fd_points_detect, Harris, 640x480, batch 1 (BASELINE configs[1]), 200 calls
  --shape northstar  fd_points_response (per-pixel kernel alone), 1920x1080 batch 256, 10 calls
                     (--kind shi_tomasi by default: the north-star kernel)
  --shape fast720    fd_points_detect, FAST, 1280x720 batch 64 (BASELINE configs[2]), 10 calls
  --shape fastbrief  the same + BRIEF-256 on the detected keypoints (fd_brief_compute), 10 calls
  --shape lsd        fd_lsd_map (dense) and fd_lsd_lines (compact map + host stage), 1920x1080 batch 256,
                     64-px checker + noise (BASELINE configs[3]), 3 calls each (--kind dense / compact: one;
                     dense_unpitched: dense maps with unpadded rows)
  --shape ties       fd_points_detect with ties="reference" on the bench tie-report frames: Harris 640x480,
                     16 seeds x 10 calls (the seeds whose frames meet a tie run k_select_reference)
  --shape nsties     the same on the north-star batch (Shi-Tomasi 1920x1080 x256), 4 calls
"""
import argparse
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

THR = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}
p = argparse.ArgumentParser()
p.add_argument("--shape", default="bench", choices=["bench", "northstar", "nsdetect", "fast720", "fast720r", "fastbrief", "lsd",
                                                   "ties", "nsties"])
p.add_argument("--kind", default=None, choices=[None, "harris", "shi_tomasi", "fast", "dense", "compact", "dense_unpitched"])
p.add_argument("--calls", type=int, default=0)
p.add_argument("--thr", type=float, default=None, help="response threshold override (e.g. 1e30: no candidates)")
a = p.parse_args()
g = torch.Generator(device="cuda")
g.manual_seed(7)


def noise(b, r, c):
    return torch.randint(0, 256, (b, r, c), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)


if a.shape == "bench":
    kind = a.kind or "harris"
    frames = noise(1, 480, 640)
    for _ in range(a.calls or 200):
        fd.detect_points(kind, frames, 200, 20, THR[kind] if a.thr is None else a.thr)
elif a.shape == "northstar":
    kind = a.kind or "shi_tomasi"
    frames = noise(256, 1080, 1920)
    cap = 1080 * 1920 if kind == "fast" else 1080 * 1920 // 2 + 64
    out = (torch.empty((256, cap), dtype=torch.float32, device="cuda"),
           torch.empty((256, cap), dtype=torch.int32, device="cuda"), torch.empty((256,), dtype=torch.int32, device="cuda"))
    for _ in range(a.calls or 10):
        fd.point_response(kind, frames, THR[kind] if a.thr is None else a.thr, out=out)
elif a.shape == "lsd":
    kind = "lsd"
    rows, cols, n = 1080, 1920, 256
    r = torch.arange(rows, device="cuda").view(1, rows, 1) // 64
    c = torch.arange(cols, device="cuda").view(1, 1, cols) // 64
    base = torch.where(((r + c) % 2) == 1, 180, 60)
    frames = (base + torch.randint(-10, 11, (n, rows, cols), generator=g, device="cuda", dtype=torch.int32)).clamp(0, 255).to(torch.uint8)
    flat = None
    if a.kind == "dense_unpitched":  # the dense maps without row padding (misaligned row stores)
        mr, mc = rows - 1, cols - 1
        flat = (torch.empty((n, mr, mc), device="cuda"), torch.empty((n, mr, mc), device="cuda"),
                torch.empty((n, mr, mc), dtype=torch.uint8, device="cuda"),
                torch.empty((n, mr * mc), dtype=torch.int32, device="cuda"), torch.empty((n,), dtype=torch.int64, device="cuda"))
    for _ in range(a.calls or 3):  # --kind dense / compact: one of the two only
        if a.kind == "dense_unpitched":
            fd.lsd_map(frames, out=flat)
            continue
        if a.kind != "compact":
            fd.lsd_map(frames)
        if a.kind != "dense":
            fd.lsd_lines(frames, max_lines=2048)
elif a.shape == "nsdetect":  # north-star shape through fd_points_detect (K1 with the selection histogram)
    kind = a.kind or "shi_tomasi"
    frames = noise(256, 1080, 1920)
    for _ in range(a.calls or 10):
        try:
            fd.detect_points(kind, frames, 200, 20, THR[kind], ties="raster")
        except Exception as e:  # (diagnostic builds that break the selection still time the kernels)
            print("detect:", e)
elif a.shape in ("ties", "nsties"):  # bench.tie_report's frames (bench.make_frames)
    import bench  # noqa: E402
    if a.shape == "ties":
        kind = a.kind or "harris"
        pool = [bench.make_frames(torch, "noise", 1, 480, 640, 1234 + 7919 * i, "cuda") for i in range(16)]
        for f in pool:
            for _ in range(a.calls or 10):
                fd.detect_points(kind, f, 200, 20, THR[kind], ties="reference")
    else:
        kind = a.kind or "shi_tomasi"
        f = bench.make_frames(torch, "noise", 256, 1080, 1920, 99, "cuda")
        for _ in range(a.calls or 4):
            fd.detect_points(kind, f, 200, 20, THR[kind], ties="reference")
elif a.shape == "fast720r":  # the FAST kernel alone (fd_points_response: no selection histogram)
    kind = "fast"
    frames = noise(64, 720, 1280)
    cap = 720 * 1280
    out = (torch.empty((64, cap), dtype=torch.float32, device="cuda"),
           torch.empty((64, cap), dtype=torch.int32, device="cuda"), torch.empty((64,), dtype=torch.int32, device="cuda"))
    for _ in range(a.calls or 10):
        fd.point_response(kind, frames, THR[kind], out=out)
elif a.shape == "fastbrief":  # BASELINE configs[2]: FAST detect + BRIEF-256 on the device output
    kind = "fast"
    frames = noise(64, 720, 1280)
    for _ in range(a.calls or 10):
        res = fd.detect_points(kind, frames, 200, 20, THR[kind])
        fd.brief_compute(frames, res.xy, res.counts, length=256, half_patch_size=8)
else:
    kind = a.kind or "fast"
    frames = noise(64, 720, 1280)
    for _ in range(a.calls or 10):
        fd.detect_points(kind, frames, 200, 20, THR[kind])
torch.cuda.synchronize()
print("done", a.shape, kind)
