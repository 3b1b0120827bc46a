"""Phase timing of fd_lsd_lines at BASELINE configs[3] (1920x1080 x 256, 64-px checker + noise)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("FD_LINES_TIMING", "1")
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402

g = torch.Generator(device="cuda")
g.manual_seed(4242)
rows, cols, n = 1080, 1920, 256
r = torch.arange(rows, device="cuda").view(1, rows, 1) // 64
c = torch.arange(cols, device="cuda").view(1, 1, cols) // 64
base = torch.where(((r + c) % 2) == 1, 180, 60)
frames = (base + torch.randint(-10, 11, (n, rows, cols), generator=g, device="cuda", dtype=torch.int32)).clamp(0, 255).to(torch.uint8)
for t in [int(x) for x in (sys.argv[1:] or ["16"])]:
    for _ in range(3):
        t0 = time.perf_counter()
        segs = fd.lsd_lines(frames, max_lines=8192, threads=t)
        print(f"threads {t}: {1e3 * (time.perf_counter() - t0):.2f} ms, lines {sum(len(s) for s in segs)}", flush=True)
