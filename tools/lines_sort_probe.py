"""Probe (diagnostic): can the reference-tie-order selection (fd_points_select with caller lists in push
order, ties="reference", distance 0, need = every candidate) produce the LSD seed order -- std::sort of the
column-major valid list by gradient norm, descending (feature_line_detector.cpp:92-94) -- on the GPU, and
how fast? Frames: configs[3]'s 1920x1080 64-px checker + noise. Checks the permutation against the
oracle's std::sort (orc_lsd_sort, sort_mode 0) and prints the selection's time per batch.
usage: python3 tools/lines_sort_probe.py [batch]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from oracle import oracle as O  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 4
rows, cols = 1080, 1920
g = torch.Generator(device="cuda")
g.manual_seed(5)
r = torch.arange(rows, device="cuda").view(1, rows, 1) // 64
c = torch.arange(cols, device="cuda").view(1, 1, cols) // 64
base = torch.where(((r + c) % 2) == 1, 180, 60)
frames = (base + torch.randint(-10, 11, (batch, rows, cols), generator=g, device="cuda", dtype=torch.int32)).clamp(0, 255).to(torch.uint8)
norm, ang, val, idx, cnt = fd.lsd_map(frames)
torch.cuda.synchronize()
mr, mc = rows - 1, cols - 1
n = cnt.to(torch.int64)
cap = int(n.max().item())
idx = idx[:, :cap].contiguous()
flat = norm.contiguous().view(batch, -1)
resp = torch.gather(flat, 1, idx.clamp(min=0).to(torch.int64)).contiguous()
xs = (idx % mc).to(torch.int32).contiguous()
ys = (idx // mc).to(torch.int32).contiguous()
print(f"batch {batch}, valid per frame {n.tolist()[:4]}...", flush=True)
res = fd.select_points((resp, xs, ys, n), mr, mc, cap, min_feature_distance=0, ties="reference")
torch.cuda.synchronize()
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    res = fd.select_points((resp, xs, ys, n), mr, mc, cap, min_feature_distance=0, ties="reference")
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / reps
st = res.status.cpu().numpy() if res.status is not None else None
print(f"select_points (reference order, all {cap} candidates): {ms:.2f} ms per batch; status {None if st is None else [hex(int(v)) for v in st[:4]]}", flush=True)
xy = res.xy.cpu().numpy()
counts = res.counts.cpu().numpy()
nm = norm.contiguous().cpu().numpy()
ok = 0
for b in range(min(batch, 4)):
    k = int(n[b])
    order = (xy[b, :counts[b], 1].astype(np.int64) * mc + xy[b, :counts[b], 0].astype(np.int64)).astype(np.int32)
    ref = O.lsd_sort(nm[b].reshape(-1), idx[b, :k].cpu().numpy(), 0)
    same = counts[b] == k and np.array_equal(order, ref)
    ok += int(same)
    print(f"frame {b}: {counts[b]} / {k} features, permutation equal to std::sort: {same}", flush=True)
print("done", ok)
