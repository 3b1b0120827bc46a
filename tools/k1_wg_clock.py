"""Diagnostic (instrumented build only: `make OUT=/tmp/clk XFLAGS=-DFD_K1_CLOCKS`, then
FD_LIB_PATH=/tmp/clk/libfdhip.so, which exports fd_debug_k1_clocks): per-workgroup
s_memrealtime clocks (100 MHz) of the headline K1 (Harris 640x480 batch 1, sorted-segment detect):
entry, after the LDS histogram clear, after the tile loop, after the segment flush. Prints the spread
of workgroup starts and each phase's distribution for the last of N calls."""
import ctypes
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from feature_detector_amd import _lib  # noqa: E402

L = _lib.load()
g = torch.Generator(device="cuda")
g.manual_seed(7)
fr = torch.randint(0, 256, (1, 480, 640), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
for it in range(int(os.environ.get("CALLS", "50"))):
    fd.detect_points("harris", fr, 200, 20, 30.0, ties="raster")
torch.cuda.synchronize()
nwg = 120
buf = (ctypes.c_ulonglong * (4 * nwg))()
assert L.fd_debug_k1_clocks(buf, 4 * nwg) == 0
s = np.array(buf, dtype=np.int64).reshape(nwg, 4)
t0 = s[:, 0].min()
us = (s - t0) / 100.0  # 100 MHz ticks -> us
def q(v):
    return "min %.2f p50 %.2f max %.2f" % (np.min(v), np.median(v), np.max(v))
print("WG entry (us after first):", q(us[:, 0]))
print("clear   (entry->clr):", q(us[:, 1] - us[:, 0]))
print("tiles   (clr->tile): ", q(us[:, 2] - us[:, 1]))
print("flush   (tile->end): ", q(us[:, 3] - us[:, 2]))
print("WG end (us after first entry):", q(us[:, 3]))
