"""Batch host API over libfdhip.so: contexts, point detection, candidates, LSD map.

Inputs are numpy arrays (host memory, staged by the library) or torch CUDA/ROCm tensors (device
memory, used in place on the context's stream, which follows torch's current stream). Every call
runs the HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import FD_FAST, FD_HARRIS, FD_SHI_TOMASI, fd_point_opts

KINDS = {"harris": FD_HARRIS, "shi_tomasi": FD_SHI_TOMASI, "fast": FD_FAST}
# order of equal responses in the selection (include/fd_hip.h fd_ctx_set_tie_order)
TIES = {"raster": 0, "reference": 1}
FRAME_TIES, FRAME_RESOLVED, FRAME_UNRESOLVED, FRAME_VALUE_RANGE, FRAME_GUARD = 0x1, 0x2, 0x4, 0x40000000, 0xBE000000
FRAME_REDETECTED = 0x8  # FAST, raster order: selected a second time without the adaptive emission cut

_ctx_lock = threading.Lock()
_contexts: dict[int, "Context"] = {}


class Context:
    """One fd_ctx: a HIP stream and grow-only device workspace on one GPU (not thread-safe)."""

    def __init__(self, device: int = 0):
        L = _lib.load()
        p = ctypes.c_void_p()
        rc = L.fd_ctx_create(int(device), ctypes.byref(p))
        if rc != _lib.FD_OK:
            raise _lib.FdError(rc, f"fd_ctx_create(device={device}) failed (is a GPU visible?)")
        self.ptr = p
        self.device = int(device)

    def close(self):
        if self.ptr:
            _lib.load().fd_ctx_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int | None):
        """Run on the given hipStream_t (0 = the HIP null stream); None = the context's own stream."""
        if stream_handle is None:
            _lib.check(self.ptr, _lib.load().fd_ctx_use_own_stream(self.ptr))
        else:
            _lib.check(self.ptr, _lib.load().fd_ctx_set_stream(self.ptr, ctypes.c_void_p(int(stream_handle))))

    def synchronize(self):
        _lib.check(self.ptr, _lib.load().fd_ctx_synchronize(self.ptr))

    def reserve(self, kind: int, batch: int, rows: int, cols: int, max_prior_total: int = 0):
        _lib.check(self.ptr, _lib.load().fd_ctx_reserve(self.ptr, kind, batch, rows, cols, max_prior_total))

    def set_tie_order(self, ties: str):
        """'raster' (equal responses by raster index) or 'reference' (the reference's std::sort order)."""
        _lib.check(self.ptr, _lib.load().fd_ctx_set_tie_order(self.ptr, TIES[ties]))

    def frame_status(self, batch: int, out=None):
        """Per-frame FD_FRAME_* words of the last selection call: numpy uint32 [batch] (synchronous), or
        copied asynchronously into `out` (a device int32 tensor [batch]) on the context stream."""
        if out is not None:
            _lib.check(self.ptr, _lib.load().fd_ctx_frame_status(self.ptr, ctypes.c_void_p(out.data_ptr()), batch, 1))
            return out
        st = np.zeros((batch,), np.uint32)
        _lib.check(self.ptr, _lib.load().fd_ctx_frame_status(self.ptr, ctypes.c_void_p(st.ctypes.data), batch, 0))
        return st


def _default_device() -> int:
    return int(os.environ.get("FD_DEVICE", "0"))


def default_context(device: int | None = None) -> Context:
    """The shared context of a GPU (default: $FD_DEVICE or 0), created on first use."""
    device = _default_device() if device is None else int(device)
    with _ctx_lock:
        c = _contexts.get(device)
        if c is None:
            c = Context(device)
            _contexts[device] = c
        return c


def _is_torch_device_tensor(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def _frames(x):
    """(pointer, on_device, batch, rows, cols, keepalive) for a u8 [B,]R,C array or tensor."""
    if _is_torch_device_tensor(x):
        import torch

        if x.dtype != torch.uint8:
            raise TypeError("frames must be uint8")
        if not x.is_contiguous():
            x = x.contiguous()
        shape = tuple(x.shape)
        ptr, on_dev = x.data_ptr(), 1
    else:
        x = np.ascontiguousarray(x)
        if x.dtype != np.uint8:
            raise TypeError("frames must be uint8")
        shape = x.shape
        ptr, on_dev = x.ctypes.data, 0
    if len(shape) == 2:
        b, r, c = 1, shape[0], shape[1]
    elif len(shape) == 3:
        b, r, c = shape
    else:
        raise ValueError("frames must be [rows, cols] or [batch, rows, cols]")
    return ptr, on_dev, int(b), int(r), int(c), x


def _resolve_ctx(ctx: Context | None, *inputs) -> Context:
    """The context of a call: `ctx`, or the default context of the GPU the torch inputs live on. A
    context on another device than its inputs is an error (its workspace and stream are per device)."""
    dev = None
    for x in inputs:
        if _is_torch_device_tensor(x):
            import torch

            d = x.device.index if x.device.index is not None else torch.cuda.current_device()
            if dev is not None and d != dev:
                raise ValueError(f"inputs on different devices ({dev} and {d})")
            dev = d
    if ctx is None:
        return default_context(dev)
    if dev is not None and ctx.device != dev:
        raise ValueError(f"context is on device {ctx.device} but the inputs are on device {dev}")
    return ctx


def _bind_stream(ctx: Context, on_device: bool):
    """Device inputs run on torch's current stream of the context's device; host inputs on the
    context's own stream. (The library orders a stream switch after the previous stream's work.)"""
    if on_device:
        import torch

        ctx.set_stream(torch.cuda.current_stream(ctx.device).cuda_stream)
    else:
        ctx.set_stream(None)


def _priors(prior, batch):
    """prior: None, or a list (per frame) of (n_i, 2) float arrays of (x, y)."""
    if prior is None:
        return None, None, None
    if len(prior) != batch:
        raise ValueError("prior must have one entry per frame")
    counts = np.array([len(p) for p in prior], np.int32)
    flat = (np.concatenate([np.asarray(p, np.float32).reshape(-1, 2) for p in prior]) if counts.sum() > 0
            else np.zeros((1, 2), np.float32))
    flat = np.ascontiguousarray(flat, np.float32)
    return flat, counts, (flat, counts)


@dataclass
class DetectResult:
    xy: object  # [batch, stride, 2] float32 (numpy or torch)
    counts: object  # [batch] int32
    status: object = None  # [batch] FD_FRAME_* words (numpy uint32, or a device int32 tensor), if fetched

    def features(self, b: int) -> np.ndarray:
        xy = self.xy if isinstance(self.xy, np.ndarray) else self.xy.cpu().numpy()
        n = int(self.counts[b]) if isinstance(self.counts, np.ndarray) else int(self.counts[b].item())
        return xy[b, :n].copy()

    def frame_flags(self) -> np.ndarray:
        """Per-frame FD_FRAME_* words as numpy uint32 (synchronises a device result)."""
        if self.status is None:
            raise ValueError("status was not fetched (out= without a status tensor)")
        st = self.status if isinstance(self.status, np.ndarray) else self.status.cpu().numpy()
        return st.astype(np.uint32)

    def check(self) -> "DetectResult":
        """Raise if a frame tripped an internal guard, or was left unresolved in the reference tie order
        (FRAME_UNRESOLVED: device results carry no flags in their counts)."""
        bad = np.nonzero(self.frame_flags() & np.uint32(FRAME_GUARD | FRAME_VALUE_RANGE | FRAME_UNRESOLVED))[0]
        if len(bad):
            raise _lib.FdError(_lib.FD_ERR_HIP, f"selection flags 0x{int(self.frame_flags()[bad[0]]):x} on frame {bad[0]}")
        return self


def detect_points(kind, frames, need: int, min_feature_distance: int = 15, min_valid_response: float = 0.1,
                  prior=None, ctx: Context | None = None, out=None, ties: str | None = None) -> DetectResult:
    """FeaturePointDetector::DetectGoodFeatures on a batch (include/fd_hip.h fd_points_detect).

    Returns the NEW features per frame (x, y), in selection order, and the per-frame status words.
    ties="reference": frames whose greedy scan meets equal responses are re-selected in the
    reference's std::sort order (libstdc++'s introsort emulated on the GPU, k_select_reference), so
    every frame equals the reference's DetectGoodFeatures; asynchronous and graph-capturable once the
    workspace exists (one call of the shape first). ties="raster": equal responses by raster index;
    identical to "reference" wherever no tie reaches the scan, and FD_FRAME_TIES in the status words
    marks the frames where one did. Default (None): "reference" for host frames
    (the reference API's semantics), "raster" for torch device frames (asynchronous; check
    `frame_flags() & FRAME_TIES` or pass ties="reference" to get the reference order there too).
    With torch device frames the outputs are device tensors (on the current stream); `out` may pass
    preallocated (xy, counts) or (xy, counts, status) tensors so that repeated calls allocate nothing.
    """
    kind = KINDS[kind] if isinstance(kind, str) else int(kind)
    ptr, on_dev, b, r, c, keep = _frames(frames)
    ctx = _resolve_ctx(ctx, frames)
    _bind_stream(ctx, bool(on_dev))
    if ties is None:
        ties = "raster" if on_dev else "reference"
    ctx.set_tie_order(ties)
    opts = fd_point_opts(int(min_feature_distance), float(min_valid_response))
    pxy, pcnt, _keep2 = _priors(prior, b)
    stride = max(int(need), 1) + 1
    status = None
    if on_dev:
        import torch

        if out is None:
            xy = torch.empty((b, stride, 2), dtype=torch.float32, device=frames.device)
            cnt = torch.empty((b,), dtype=torch.int32, device=frames.device)
            status = torch.empty((b,), dtype=torch.int32, device=frames.device)
        else:
            xy, cnt = out[0], out[1]
            status = out[2] if len(out) > 2 else None
            stride = xy.shape[1]
        xy_ptr, cnt_ptr = xy.data_ptr(), cnt.data_ptr()
    else:
        xy = np.zeros((b, stride, 2), np.float32)
        cnt = np.zeros((b,), np.int32)
        xy_ptr, cnt_ptr = xy.ctypes.data, cnt.ctypes.data
    rc = _lib.load().fd_points_detect(
        ctx.ptr, kind, ctypes.c_void_p(ptr), on_dev, b, r, c, ctypes.byref(opts),
        ctypes.c_void_p(pxy.ctypes.data) if pxy is not None else None,
        ctypes.c_void_p(pcnt.ctypes.data) if pcnt is not None else None,
        int(need), ctypes.c_void_p(xy_ptr), stride, ctypes.c_void_p(cnt_ptr), on_dev)
    _lib.check(ctx.ptr, rc)
    del keep
    if on_dev:
        if status is not None:
            ctx.frame_status(b, out=status)
    else:
        status = ctx.frame_status(b)
    return DetectResult(xy, cnt, status)


def select_points(candidates, rows: int, cols: int, need: int, min_feature_distance: int = 15, prior=None,
                  ties: str | None = None, ctx: Context | None = None, out=None) -> DetectResult:
    """SelectGoodFeatures over caller-supplied candidates (fd_points_select): the ComputeCandidates
    seam of a detector whose candidates come from elsewhere (feature_point_detector.h:44).

    candidates: a list (per frame) of (resp, x, y) arrays in the order they were pushed -- host
    arrays, returns numpy results (ties default "reference"); or a tuple of torch device tensors
    (resp [B, cap] float32, x [B, cap] int32, y [B, cap] int32, counts [B] int64), returns device
    tensors asynchronously (ties default "raster"; `out` as in detect_points).
    """
    opts = fd_point_opts(int(min_feature_distance), 0.0)
    L = _lib.load()
    if isinstance(candidates, tuple) and hasattr(candidates[0], "data_ptr"):
        import torch

        resp, xs, ys, counts = candidates
        b, cap = resp.shape
        for t, dt in ((resp, torch.float32), (xs, torch.int32), (ys, torch.int32)):
            if t.dtype != dt or tuple(t.shape) != (b, cap) or not t.is_cuda or not t.is_contiguous():
                raise ValueError("device candidates: contiguous resp f32 / x, y int32 [B, cap] tensors")
        if counts.dtype != torch.int64 or tuple(counts.shape) != (b,) or not counts.is_cuda:
            raise ValueError("device candidates: counts int64 [B]")
        ctx = _resolve_ctx(ctx, resp)
        _bind_stream(ctx, True)
        ctx.set_tie_order(ties or "raster")
        pxy, pcnt, _keep2 = _priors(prior, b)
        stride = max(int(need), 1) + 1
        status = None
        if out is None:
            xy = torch.empty((b, stride, 2), dtype=torch.float32, device=resp.device)
            cnt = torch.empty((b,), dtype=torch.int32, device=resp.device)
            status = torch.empty((b,), dtype=torch.int32, device=resp.device)
        else:
            xy, cnt = out[0], out[1]
            status = out[2] if len(out) > 2 else None
            stride = xy.shape[1]
        rc = L.fd_points_select(ctx.ptr, b, rows, cols, ctypes.byref(opts), ctypes.c_void_p(resp.data_ptr()),
                                ctypes.c_void_p(xs.data_ptr()), ctypes.c_void_p(ys.data_ptr()),
                                ctypes.c_void_p(counts.data_ptr()), int(cap), 1,
                                ctypes.c_void_p(pxy.ctypes.data) if pxy is not None else None,
                                ctypes.c_void_p(pcnt.ctypes.data) if pcnt is not None else None,
                                int(need), ctypes.c_void_p(xy.data_ptr()), stride, ctypes.c_void_p(cnt.data_ptr()), 1)
        _lib.check(ctx.ptr, rc)
        if status is not None:
            ctx.frame_status(b, out=status)
        return DetectResult(xy, cnt, status)
    b = len(candidates)
    counts = np.array([len(c[0]) for c in candidates], np.int64)
    cap = max(int(counts.max()) if b else 0, 1)
    resp = np.zeros((b, cap), np.float32)
    xs = np.zeros((b, cap), np.int32)
    ys = np.zeros((b, cap), np.int32)
    for i, (r_, x_, y_) in enumerate(candidates):
        n = counts[i]
        if len(x_) != n or len(y_) != n:
            raise ValueError(f"frame {i}: resp, x and y differ in length")
        resp[i, :n], xs[i, :n], ys[i, :n] = r_, x_, y_
    ctx = _resolve_ctx(ctx)
    _bind_stream(ctx, False)
    ctx.set_tie_order(ties or "reference")
    pxy, pcnt, _keep2 = _priors(prior, b)
    stride = max(int(need), 1) + 1
    xy = np.zeros((b, stride, 2), np.float32)
    cnt = np.zeros((b,), np.int32)
    rc = L.fd_points_select(ctx.ptr, b, rows, cols, ctypes.byref(opts), ctypes.c_void_p(resp.ctypes.data),
                            ctypes.c_void_p(xs.ctypes.data), ctypes.c_void_p(ys.ctypes.data),
                            ctypes.c_void_p(counts.ctypes.data), cap, 0,
                            ctypes.c_void_p(pxy.ctypes.data) if pxy is not None else None,
                            ctypes.c_void_p(pcnt.ctypes.data) if pcnt is not None else None,
                            int(need), ctypes.c_void_p(xy.ctypes.data), stride, ctypes.c_void_p(cnt.ctypes.data), 0)
    _lib.check(ctx.ptr, rc)
    return DetectResult(xy, cnt, ctx.frame_status(b))


def point_response(kind, frames, min_valid_response: float = 0.1, out=None, ctx: Context | None = None,
                   append: bool = False):
    """The per-pixel stage alone (fd_points_response) on torch device frames [B, R, C].

    Returns (resp, idx, counts): resp float32 [B, cap], idx int32 [B, cap] (raster index), in
    unspecified order, counts int32 [B]. Asynchronous on torch's current stream. append=True
    (fd_points_response_append, needs out=) keeps the counts in out and appends after them, so the
    call is the per-pixel kernel alone (no count reset).
    """
    import torch

    kind = KINDS[kind] if isinstance(kind, str) else int(kind)
    ptr, on_dev, b, r, c, keep = _frames(frames)
    if not on_dev:
        raise TypeError("point_response takes device frames")
    ctx = _resolve_ctx(ctx, frames)
    _bind_stream(ctx, True)
    cap = r * c if kind == FD_FAST else r * c // 2 + 64
    if out is None:
        resp = torch.empty((b, cap), dtype=torch.float32, device=frames.device)
        idx = torch.empty((b, cap), dtype=torch.int32, device=frames.device)
        counts = torch.empty((b,), dtype=torch.int32, device=frames.device)
    else:
        resp, idx, counts = out
        cap = resp.shape[1]
    if append and out is None:
        raise ValueError("append=True needs out=(resp, idx, counts)")
    opts = fd_point_opts(15, float(min_valid_response))
    L = _lib.load()
    fn = L.fd_points_response_append if append else L.fd_points_response
    rc = fn(ctx.ptr, kind, ctypes.c_void_p(ptr), b, r, c, ctypes.byref(opts),
            ctypes.c_void_p(resp.data_ptr()), ctypes.c_void_p(idx.data_ptr()), int(cap),
            ctypes.c_void_p(counts.data_ptr()))
    _lib.check(ctx.ptr, rc)
    del keep
    return resp, idx, counts


def point_candidates(kind, frames, min_feature_distance: int = 15, min_valid_response: float = 0.1, prior=None,
                     cap: int | None = None, response_map: bool = False, ctx: Context | None = None):
    """The ComputeCandidates seam (fd_points_candidates): raster-ordered candidates per frame.

    Host (numpy) frames only. Returns a list of (resp, x, y) arrays per frame, and the response map
    [batch, rows, cols] if requested.
    """
    kind = KINDS[kind] if isinstance(kind, str) else int(kind)
    ptr, on_dev, b, r, c, keep = _frames(frames)
    if on_dev:
        raise TypeError("point_candidates takes host frames")
    ctx = _resolve_ctx(ctx, frames)
    _bind_stream(ctx, False)
    opts = fd_point_opts(int(min_feature_distance), float(min_valid_response))
    pxy, pcnt, _keep2 = _priors(prior, b)
    if cap is None:
        cap = r * c if kind == FD_FAST else r * c // 2 + 16
    resp = np.zeros((b, max(cap, 1)), np.float32)
    xs = np.zeros((b, max(cap, 1)), np.int32)
    ys = np.zeros((b, max(cap, 1)), np.int32)
    counts = np.zeros((b,), np.int64)
    rmap = np.zeros((b, r, c), np.float32) if response_map else None
    rc = _lib.load().fd_points_candidates(
        ctx.ptr, kind, ctypes.c_void_p(ptr), 0, b, r, c, ctypes.byref(opts),
        ctypes.c_void_p(pxy.ctypes.data) if pxy is not None else None,
        ctypes.c_void_p(pcnt.ctypes.data) if pcnt is not None else None,
        ctypes.c_void_p(resp.ctypes.data), ctypes.c_void_p(xs.ctypes.data), ctypes.c_void_p(ys.ctypes.data),
        int(cap), ctypes.c_void_p(counts.ctypes.data),
        ctypes.c_void_p(rmap.ctypes.data) if rmap is not None else None, 0)
    _lib.check(ctx.ptr, rc)
    del keep
    out = [(resp[i, :counts[i]].copy(), xs[i, :counts[i]].copy(), ys[i, :counts[i]].copy()) for i in range(b)]
    return (out, rmap) if response_map else out


def lsd_map(frames, min_norm: float = 20.0, cap: int | None = None, ctx: Context | None = None, out=None):
    """ComputeLineLevelAngleMap (fd_lsd_map / fd_lsd_map_pitched).

    Host (numpy) frames: returns per frame (norm, angle, valid, valid_idx_colmajor); maps are
    (rows-1, cols-1). Torch device frames: returns device tensors (norm [B, R-1, C-1] f32, angle f32,
    valid u8, valid_idx int32 [B, cap], counts int64 [B]), asynchronous on torch's current stream;
    the maps are views of storage whose rows are padded to 16 entries (aligned row stores); `out` may
    pass them preallocated (graph capture), contiguous or as such row-padded views sharing one row
    pitch; any of norm/angle/valid may be None to skip.
    """
    ptr, on_dev, b, r, c, keep = _frames(frames)
    ctx = _resolve_ctx(ctx, frames)
    mr, mc = r - 1, c - 1
    cap = mr * mc if cap is None else cap
    if on_dev:
        import torch

        if out is None:
            dev = frames.device
            pitch = (mc + 15) // 16 * 16
            out = (torch.empty((b, mr, pitch), dtype=torch.float32, device=dev)[..., :mc],
                   torch.empty((b, mr, pitch), dtype=torch.float32, device=dev)[..., :mc],
                   torch.empty((b, mr, pitch), dtype=torch.uint8, device=dev)[..., :mc],
                   torch.empty((b, max(cap, 1)), dtype=torch.int32, device=dev),
                   torch.empty((b,), dtype=torch.int64, device=dev))
        norm, ang, val, idx, cnt = out
        pitch = None
        for t in (norm, ang, val):
            if t is None:
                continue
            if tuple(t.shape) != (b, mr, mc) or t.stride(2) != 1 or t.stride(0) != mr * t.stride(1):
                raise ValueError(f"lsd_map: maps must be [{b}, {mr}, {mc}] with unit column stride and rows "
                                 "packed at one pitch")
            if pitch not in (None, t.stride(1)):
                raise ValueError("lsd_map: norm / angle / valid must share one row pitch")
            pitch = t.stride(1)
        pitch = mc if pitch is None else pitch
        cap = idx.shape[1]
        _bind_stream(ctx, True)

        def p(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        rc = _lib.load().fd_lsd_map_pitched(ctx.ptr, ctypes.c_void_p(ptr), 1, b, r, c, float(min_norm), p(norm),
                                            p(ang), p(val), int(pitch), p(idx), int(cap), p(cnt), 1)
        _lib.check(ctx.ptr, rc)
        del keep
        return out
    _bind_stream(ctx, False)
    norm = np.zeros((b, mr, mc), np.float32)
    ang = np.zeros((b, mr, mc), np.float32)
    val = np.zeros((b, mr, mc), np.uint8)
    idx = np.zeros((b, max(cap, 1)), np.int32)
    cnt = np.zeros((b,), np.int64)
    rc = _lib.load().fd_lsd_map(ctx.ptr, ctypes.c_void_p(ptr), 0, b, r, c, float(min_norm),
                                ctypes.c_void_p(norm.ctypes.data), ctypes.c_void_p(ang.ctypes.data),
                                ctypes.c_void_p(val.ctypes.data), ctypes.c_void_p(idx.ctypes.data), int(cap),
                                ctypes.c_void_p(cnt.ctypes.data), 0)
    _lib.check(ctx.ptr, rc)
    del keep
    return [(norm[i], ang[i], val[i], idx[i, :cnt[i]].copy()) for i in range(b)]


# FeatureLineDetector::Options defaults (feature_line_detector.h:40-45); kDegToRad = kPai / 180 in float.
LSD_TOL_RAD = float(np.float32(22.5) * (np.float32(3.14159265358979323846) / np.float32(180.0)))


def lsd_lines(frames, needed: int = 1, min_norm: float = 20.0, tol_rad: float = LSD_TOL_RAD, min_length: float = 20.0,
              min_inlier: float = 0.6, max_lines: int = 4096, threads: int = 0, ctx: Context | None = None):
    """FeatureLineDetector::DetectGoodFeatures for a batch (fd_lsd_lines): GPU level-line map (compact
    lists), region growing and rectangle fitting on `threads` host threads (0: all, capped by
    OMP_NUM_THREADS). frames: numpy [B, R, C] / [R, C] u8 or a torch device tensor.

    Returns a list over frames of float32 arrays [n, 12] (start x, y, end x, y, center x, y, length,
    width, angle, dir x, y, inlier ratio); columns 0-3 are the reference's Vec4 features."""
    ptr, on_dev, b, r, c, keep = _frames(frames)
    ctx = _resolve_ctx(ctx, frames)
    _bind_stream(ctx, on_dev)
    opts = _lib.fd_lsd_opts(float(min_norm), float(tol_rad), float(min_length), float(min_inlier))
    out = np.empty((b, max(max_lines, 1), _lib.LSD_RECT_FLOATS), np.float32)
    cnt = np.zeros((b,), np.int32)
    rc = _lib.load().fd_lsd_lines(ctx.ptr, ctypes.c_void_p(ptr), 1 if on_dev else 0, b, r, c, ctypes.byref(opts),
                                  int(needed), ctypes.c_void_p(out.ctypes.data), int(max_lines),
                                  ctypes.c_void_p(cnt.ctypes.data), int(threads))
    _lib.check(ctx.ptr, rc)
    del keep
    if (cnt > max_lines).any():
        raise _lib.FdError(_lib.FD_ERR_CAPACITY, f"max_lines={max_lines} < {int(cnt.max())} segments found")
    return [out[i, :cnt[i]].copy() for i in range(b)]
