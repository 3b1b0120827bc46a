"""Steered BRIEF descriptors over the C ABI (fd_brief_compute), SURVEY §8 row f1.

Mirrors feature_detector::BriefDescriptor (descriptor_brief.h:14-37) for batches: Options kLength /
kHalfPatchSize, plus the float-coordinate sampler the reference takes from its un-vendored
GrayImage (bilinear by default, truncation selectable; DESIGN.md: parity unpinned for the sampled
bits, exact for everything before them). Keypoints are (x, y) = (col, row), the layout
detect_points returns, so a device-side detect -> describe chain stays on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import FD_SAMPLE_BILINEAR, FD_SAMPLE_TRUNCATE, fd_brief_opts
from .points import Context, _bind_stream, _frames, _is_torch_device_tensor, _resolve_ctx

SAMPLERS = {"bilinear": FD_SAMPLE_BILINEAR, "truncate": FD_SAMPLE_TRUNCATE}


def brief_compute(frames, uv, counts=None, length: int = 256, half_patch_size: int = 8, sampler="bilinear",
                  with_valid: bool = False, out=None, ctx: Context | None = None):
    """Descriptor<BriefType>::Compute (descriptor.h:27-40) for a batch.

    frames: u8 [B, R, C] or [R, C]; uv: float32 [B, S, 2] or [S, 2] keypoints (x, y); counts: int32 [B]
    keypoints per frame (None = S each). Host (numpy) frames/uv give numpy outputs; torch device uv
    (with device frames) gives torch outputs, asynchronous on torch's current stream.
    Returns bits uint32 [B, S, ceil(length/32)] (bit i of a descriptor = bit i%32 of word i/32;
    slots >= counts[b] are left zero), and valid uint8 [B, S] if with_valid. Device path only: out=
    a preallocated int32 [B, S, words] tensor (slots >= counts[b] then keep their contents), so the
    call is the kernel alone (graph-capturable without an allocation or fill).
    """
    smp = SAMPLERS[sampler] if isinstance(sampler, str) else int(sampler)
    fptr, f_on_dev, b, r, c, keep_f = _frames(frames)
    ctx = _resolve_ctx(ctx, frames, uv)
    nw = (int(length) + 31) // 32
    opts = fd_brief_opts(int(length), int(half_patch_size), smp)
    if _is_torch_device_tensor(uv):
        import torch

        uv_t = uv.to(torch.float32).contiguous()
        if uv_t.dim() == 2:
            uv_t = uv_t.unsqueeze(0)
        if uv_t.shape[0] != b or uv_t.shape[2] != 2:
            raise ValueError("uv must be [batch, S, 2] matching frames")
        s = int(uv_t.shape[1])
        cnt_t = None if counts is None else counts.to(torch.int32).contiguous()
        if out is not None:
            if tuple(out.shape) != (b, s, nw) or out.dtype != torch.int32 or not out.is_contiguous():
                raise ValueError(f"out must be a contiguous int32 tensor of shape {(b, s, nw)}")
            bits = out
        else:
            bits = torch.zeros((b, s, nw), dtype=torch.int32, device=uv_t.device)
        valid = torch.zeros((b, s), dtype=torch.uint8, device=uv_t.device) if with_valid else None
        _bind_stream(ctx, True)
        rc = _lib.load().fd_brief_compute(
            ctx.ptr, ctypes.c_void_p(fptr), f_on_dev, b, r, c, ctypes.byref(opts), ctypes.c_void_p(uv_t.data_ptr()),
            ctypes.c_void_p(cnt_t.data_ptr()) if cnt_t is not None else None, s, ctypes.c_void_p(bits.data_ptr()),
            ctypes.c_void_p(valid.data_ptr()) if valid is not None else None, 1)
        _lib.check(ctx.ptr, rc)
        del keep_f
        return (bits, valid) if with_valid else bits
    uv_h = np.asarray(uv, np.float32)
    if uv_h.ndim == 2:
        uv_h = uv_h[None]
    uv_h = np.ascontiguousarray(uv_h)
    if uv_h.shape[0] != b or uv_h.shape[2] != 2:
        raise ValueError("uv must be [batch, S, 2] matching frames")
    s = int(uv_h.shape[1])
    cnt_h = None if counts is None else np.ascontiguousarray(np.asarray(counts, np.int32).reshape(b))
    bits = np.zeros((b, s, nw), np.uint32)
    valid = np.zeros((b, s), np.uint8) if with_valid else None
    _bind_stream(ctx, bool(f_on_dev))
    rc = _lib.load().fd_brief_compute(
        ctx.ptr, ctypes.c_void_p(fptr), f_on_dev, b, r, c, ctypes.byref(opts), ctypes.c_void_p(uv_h.ctypes.data),
        ctypes.c_void_p(cnt_h.ctypes.data) if cnt_h is not None else None, s, ctypes.c_void_p(bits.ctypes.data),
        ctypes.c_void_p(valid.ctypes.data) if valid is not None else None, 0)
    _lib.check(ctx.ptr, rc)
    del keep_f
    return (bits, valid) if with_valid else bits


def unpack_bits(bits, length: int) -> np.ndarray:
    """[..., words] uint32 -> [..., length] bool (BriefType = std::vector<bool>, descriptor_brief.h:10)."""
    w = np.asarray(bits).astype(np.uint32)
    idx = np.arange(length)
    return ((w[..., idx >> 5] >> (idx & 31).astype(np.uint32)) & 1).astype(bool)


def to_float(bits, length: int) -> np.ndarray:
    """Descriptor::Compute's std::vector<Vec> overload: bit -> +1.0f / -1.0f (descriptor.h:50-53)."""
    return np.where(unpack_bits(bits, length), np.float32(1.0), np.float32(-1.0)).astype(np.float32)
