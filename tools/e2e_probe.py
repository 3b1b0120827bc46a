"""Where the per-frame host call goes (bench `end_to_end_host_frames`): the headline workload (Harris,
640x480, dist 20, need 200, thr 30) through the layers of a host-frame call, each timed alone over
~1 s of back-to-back calls on the GPU box. Prints one line per layer (microseconds per call)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import feature_detector_amd as fd  # noqa: E402
from feature_detector_amd import _lib  # noqa: E402

R, C, NEED, DIST, THR = 480, 640, 200, 20, 30.0
rng = np.random.default_rng(5)
frames = rng.integers(0, 256, (16, R, C), dtype=np.uint8)
L = _lib.load()
ctx = fd.default_context()
ctx.set_stream(None)
ctx.set_tie_order("raster")
opts = _lib.fd_point_opts(DIST, THR)
stride = NEED + 1
xy = np.zeros((1, stride, 2), np.float32)
cnt = np.zeros((1,), np.int32)
st = np.zeros((1,), np.uint32)
dptr = ctypes.c_void_p()


def bench(name, fn, secs=1.0):
    for _ in range(20):
        fn(0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        fn(n)
        n += 1
    us = (time.perf_counter() - t0) / n * 1e6
    print(f"{name:58s} {us:9.1f} us/call", flush=True)


def detect_host(i):
    rc = L.fd_points_detect(ctx.ptr, 0, ctypes.c_void_p(frames[i % 16].ctypes.data), 0, 1, R, C, ctypes.byref(opts),
                            None, None, NEED, ctypes.c_void_p(xy.ctypes.data), stride, ctypes.c_void_p(cnt.ctypes.data), 0)
    assert rc == 0


def stage(i):
    rc = L.fd_ctx_stage(ctx.ptr, ctypes.c_void_p(frames[i % 16].ctypes.data), R * C, ctypes.byref(dptr))
    assert rc == 0


def detect_staged_host_out(i):
    rc = L.fd_points_detect(ctx.ptr, 0, dptr, 1, 1, R, C, ctypes.byref(opts), None, None, NEED,
                            ctypes.c_void_p(xy.ctypes.data), stride, ctypes.c_void_p(cnt.ctypes.data), 0)
    assert rc == 0


def status(i):
    rc = L.fd_ctx_frame_status(ctx.ptr, ctypes.c_void_p(st.ctypes.data), 1, 0)
    assert rc == 0


stage(0)
bench("fd.detect_points (python, host frame, ties=raster)",
      lambda i: fd.detect_points("harris", frames[i % 16], NEED, DIST, THR, ties="raster"))
bench("fd_points_detect (ctypes, host frame, host outputs)", detect_host)
bench("  fd_ctx_stage (H2D of one frame + sync)", stage)
bench("  fd_points_detect (staged frame, host outputs)", detect_staged_host_out)
bench("  fd_ctx_frame_status (host dst, sync)", status)
bench("  fd_ctx_use_own_stream + set_tie_order", lambda i: (ctx.set_stream(None), ctx.set_tie_order("raster")))
bench("C++ drop-in: stage + detect + status (as the class)", lambda i: (stage(i), detect_staged_host_out(i)))
