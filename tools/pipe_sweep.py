"""Diagnostic: headline serving pipeline (bench.run_pipelined) with 1..4 contexts/streams."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
import feature_detector_amd as fd

fd.load()
dev = torch.device("cuda", 0)
for n in (1, 2, 3, 4, 6):
    ms, fr = bench.run_pipelined(torch, fd, dev, "harris", 480, 640, 200, 20, "noise", seed=5, nctx=n)
    print(f"nctx={n}: {ms * 1e3:.2f} us/frame, {480 * 640 / (ms * 1e-3) / 1e6:.0f} Mpix/s", flush=True)
