"""Pipelined host-frame ingest over fd_ingest_* (fd_ingest.cpp).

`depth` pinned slots of `batch` frames: write frames into `frames(slot)` (a numpy view of pinned host
memory), `submit(slot)` (upload on the ingest's copy stream, detection and feature copy-back on the
context stream; returns at once), `wait(slot)` -> per-frame feature arrays. Uploads of one slot overlap
the detection of the previous one. Mirrors what a reference caller does per image
(Visualizor2D::LoadImage then DetectGoodFeatures, test_feature_point_detector.cpp:104-110), batched.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import fd_point_opts
from .points import KINDS, Context


class Ingest:
    def __init__(self, detector: str, rows: int, cols: int, batch: int = 16, depth: int = 3, need: int = 200,
                 min_feature_distance: int = 20, min_valid_response: float | None = None, device: int = 0):
        self.kind = KINDS[detector]
        thr = {"harris": 30.0, "shi_tomasi": 40.0, "fast": 10.0}[detector] if min_valid_response is None else min_valid_response
        self.opts = fd_point_opts(int(min_feature_distance), float(thr))
        self.rows, self.cols, self.batch, self.depth, self.need = int(rows), int(cols), int(batch), int(depth), int(need)
        self.stride = self.need + 1
        self.ctx = Context(device)  # its own context: the ingest owns the stream order of its detections
        L = _lib.load()
        p = ctypes.c_void_p()
        _lib.check(self.ctx.ptr, L.fd_ingest_create(self.ctx.ptr, self.kind, self.batch, self.rows, self.cols,
                                                    self.depth, self.need, self.stride, ctypes.byref(p)))
        self.ptr = p
        n = self.batch * self.rows * self.cols
        self._views = []
        for s in range(self.depth):
            addr = L.fd_ingest_frames(self.ptr, s)
            buf = (ctypes.c_uint8 * n).from_address(addr)
            self._views.append(np.frombuffer(buf, np.uint8).reshape(self.batch, self.rows, self.cols))

    def frames(self, slot: int) -> np.ndarray:
        """Pinned [batch, rows, cols] u8 view of the slot's frames (write them before submit)."""
        return self._views[slot]

    def submit(self, slot: int) -> None:
        _lib.check(self.ctx.ptr, _lib.load().fd_ingest_submit(self.ptr, int(slot), ctypes.byref(self.opts)))

    def wait(self, slot: int) -> list[np.ndarray]:
        """The slot's new features per frame ([n, 2] float32 (x, y), copies)."""
        xy, cnt = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(self.ctx.ptr, _lib.load().fd_ingest_wait(self.ptr, int(slot), ctypes.byref(xy), ctypes.byref(cnt)))
        counts = np.ctypeslib.as_array(ctypes.cast(cnt, ctypes.POINTER(ctypes.c_int32)), (self.batch,))
        pts = np.ctypeslib.as_array(ctypes.cast(xy, ctypes.POINTER(ctypes.c_float)), (self.batch, self.stride, 2))
        return [pts[b, : int(counts[b])].copy() for b in range(self.batch)]

    def close(self):
        if getattr(self, "ptr", None):
            _lib.load().fd_ingest_destroy(self.ptr)
            self.ptr = None
        if getattr(self, "ctx", None) is not None:
            self.ctx.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------------------ PNG front end (f4)
def png_info(data: bytes):
    """(rows, cols, channels) of a PNG stream (fd_png_info)."""
    L = _lib.load()
    r, c, ch = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    rc = L.fd_png_info(data, len(data), ctypes.byref(r), ctypes.byref(c), ctypes.byref(ch))
    if rc:
        raise _lib.FdError(rc, "not a supported PNG (8-bit gray / gray+alpha / RGB / RGBA, no interlace)")
    return r.value, c.value, ch.value


def load_png(path_or_bytes) -> np.ndarray:
    """One PNG as a gray u8 image [rows, cols] (fd_png_decode): what the reference's
    Visualizor2D::LoadImage hands DetectGoodFeatures (colour -> gray: BT.601 fixed point, unpinned)."""
    data = bytes(path_or_bytes) if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    rows, cols, _ = png_info(data)
    out = np.empty((rows, cols), np.uint8)
    r, c = ctypes.c_int32(), ctypes.c_int32()
    rc = _lib.load().fd_png_decode(data, len(data), ctypes.c_void_p(out.ctypes.data), out.size, ctypes.byref(r),
                                   ctypes.byref(c))
    if rc:
        raise _lib.FdError(rc, "PNG decode failed")
    return out


def png_frames(images, threads: int = 0, ctx: Context | None = None, out=None):
    """A batch of same-size PNG streams (bytes) -> device gray frames, a torch uint8 tensor
    [n, rows, cols] on the context's device (fd_png_frames: host decode threads, one upload, colour ->
    gray on the GPU), stream-ordered on torch's current stream."""
    import torch

    from .points import _bind_stream, default_context

    images = [bytes(x) for x in images]
    rows, cols, _ = png_info(images[0])
    ctx = ctx or default_context(torch.cuda.current_device())
    _bind_stream(ctx, True)
    n = len(images)
    if out is None:
        out = torch.empty((n, rows, cols), dtype=torch.uint8, device=f"cuda:{ctx.device}")
    elif (tuple(out.shape) != (n, rows, cols) or out.dtype != torch.uint8 or out.device.type != "cuda"
          or out.device.index != ctx.device or not out.is_contiguous()):
        raise ValueError(f"png_frames: out must be a contiguous uint8 cuda:{ctx.device} tensor of shape "
                         f"{(n, rows, cols)}, got {tuple(out.shape)} {out.dtype} on {out.device}")
    bufs = (ctypes.c_char_p * n)(*images)
    lens = (ctypes.c_size_t * n)(*[len(x) for x in images])
    rc = _lib.load().fd_png_frames(ctx.ptr, ctypes.cast(bufs, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p), n,
                                   rows, cols, ctypes.c_void_p(out.data_ptr()), int(threads))
    _lib.check(ctx.ptr, rc)
    return out
