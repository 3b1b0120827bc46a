"""Diagnostic: LSD map batch time (1920x1080 x 256 checker frames) under env-selected variants,
run under rocprofv3 --kernel-trace for the per-kernel split. usage: lsd_probe.py VAR=val,... ..."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import feature_detector_amd as fd
import bench
dev = torch.device("cuda:0")
frames = bench.make_frames(torch, "checker", 256, 1080, 1920, 4242, dev, period=64)
out = fd.lsd_map(frames)
torch.cuda.synchronize()
for spec in sys.argv[1:]:
    for kv in spec.split(","):
        k, v = kv.split("=")
        os.environ[k] = v
    ms = bench.graph_time_ms(torch, lambda: fd.lsd_map(frames, out=out), 5)
    print(spec, "%.4f ms" % ms, flush=True)
