"""SuperPoint keypoints + descriptors: the network in PyTorch-ROCm, the
post-processing in the HIP kernels behind fd_nn_select / fd_nn_descriptors.

Mirrors feature_detector::NNFeaturePointDetector (src/nn_feature_point_detector/
nn_feature_point_detector.h:12-86) for the kSuperpointHeatmap model:
  Initialize()                          nn_feature_point_detector.cpp:10-57 (network + one warm-up run)
  DetectGoodFeaturesWithDescriptor()    nn_feature_point_detector_superpoint.cpp:8-77
    InferenceSession                    -> SuperPointNet (fp16 convs through MIOpen, fp32 heatmap)
    CreateMask + candidates + selection -> fd_nn_select (GPU, std::multimap order)
    ExtractDescriptorsForSelectedFeatures -> fd_nn_descriptors (GPU bilinear sampling)

The reference loads trained ONNX models (onnx_models/superpoint.onnx) that are not available here
(.MISSING_LARGE_BLOBS), and ONNX Runtime is absent: the network is the published SuperPoint
architecture with seeded random weights, so keypoints from it are meaningful for throughput only.
The post-processing is bit-exact to the oracle's restatement on any given network output. The
kSuperpointNms / DISK variants are not provided (their in-graph NMS / UNet need the missing models).
"""
from __future__ import annotations

import os

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import fd_nn_opts
from .points import Context, _bind_stream, _is_torch_device_tensor, _resolve_ctx


@dataclass
class Options:
    """NNFeaturePointDetector::Options (nn_feature_point_detector.h:22-31)."""
    kInvalidBoundary: int = 3
    kMinFeatureDistance: int = 15
    kMaxImageRows: int = 480
    kMaxImageCols: int = 752
    kMaxNumberOfDetectedFeatures: int = 240
    kMinResponse: float = 0.1
    kModelType: str = "kSuperpointHeatmap"
    kComputeDescriptors: bool = False


def _opts(o: Options, max_response: float = 1.0) -> fd_nn_opts:
    return fd_nn_opts(int(o.kInvalidBoundary), int(o.kMinFeatureDistance), int(o.kMaxNumberOfDetectedFeatures),
                      float(o.kMinResponse), float(max_response))


def nn_select(heat, options: Options | None = None, prior=None, out=None, ctx: Context | None = None,
              max_response: float = 1.0):
    """fd_nn_select on heatmaps [B, H, W] float32 (numpy, or a torch device tensor -> device outputs).

    max_response: declared upper bound of the heatmap (1.0: softmax probabilities); float('inf') for
    arbitrary maps (coarser selection keys). A value above it fails the call.
    Returns (xy [B, max+1, 2] float32, counts [B] int32): new features per frame, selection order.
    prior: None or a list (per frame) of (n_i, 2) float arrays of (x, y), host memory.
    """
    o = options or Options()
    ctx = _resolve_ctx(ctx, heat)
    opts = _opts(o, max_response)
    on_dev = _is_torch_device_tensor(heat)
    if on_dev:
        import torch

        heat = heat.to(torch.float32).contiguous()
        ptr = heat.data_ptr()
    else:
        heat = np.ascontiguousarray(heat, np.float32)
        ptr = heat.ctypes.data
    if heat.ndim == 2:
        heat = heat[None]
    b, r, c = (int(v) for v in heat.shape)
    stride = max(int(o.kMaxNumberOfDetectedFeatures), 1) + 1
    pflat, pcnt = None, None
    if prior is not None:
        if len(prior) != b:
            raise ValueError("prior must have one entry per frame")
        pcnt = np.array([len(p) for p in prior], np.int32)
        pflat = (np.ascontiguousarray(np.concatenate([np.asarray(p, np.float32).reshape(-1, 2) for p in prior]))
                 if pcnt.sum() > 0 else np.zeros((1, 2), np.float32))
    if on_dev:
        import torch

        if out is None:
            out = (torch.empty((b, stride, 2), dtype=torch.float32, device=heat.device),
                   torch.empty((b,), dtype=torch.int32, device=heat.device))
        xy, cnt = out
        stride = xy.shape[1]
        xy_p, cnt_p = xy.data_ptr(), cnt.data_ptr()
    else:
        xy = np.zeros((b, stride, 2), np.float32)
        cnt = np.zeros((b,), np.int32)
        xy_p, cnt_p = xy.ctypes.data, cnt.ctypes.data
    _bind_stream(ctx, on_dev)
    rc = _lib.load().fd_nn_select(
        ctx.ptr, ctypes.c_void_p(ptr), 1 if on_dev else 0, b, r, c, ctypes.byref(opts),
        ctypes.c_void_p(pflat.ctypes.data) if pflat is not None else None,
        ctypes.c_void_p(pcnt.ctypes.data) if pcnt is not None else None, ctypes.c_void_p(xy_p), int(stride),
        ctypes.c_void_p(cnt_p), 1 if on_dev else 0)
    _lib.check(ctx.ptr, rc)
    return xy, cnt


def nn_descriptors(desc_map, xy, counts=None, out=None, ctx: Context | None = None):
    """fd_nn_descriptors: desc_map [B, C, h, w] float32, xy [B, S, 2] -> descriptors [B, S, C].

    Host arrays give numpy outputs; torch device tensors give device outputs (current stream)."""
    ctx = _resolve_ctx(ctx, desc_map, xy)
    if _is_torch_device_tensor(desc_map):
        import torch

        m = desc_map.to(torch.float32)
        b, ch, h, w = (int(v) for v in m.shape)
        # a channels-last map (the network's output) is read in place; anything else as NCHW
        if m.is_contiguous(memory_format=torch.channels_last) and not m.is_contiguous():
            layout = 1
        else:
            m, layout = m.contiguous(), 0
        xy_t = xy.to(torch.float32).contiguous()
        s = int(xy_t.shape[1])
        cnt_t = None if counts is None else counts.to(torch.int32).contiguous()
        res = out if out is not None else torch.zeros((b, s, ch), dtype=torch.float32, device=m.device)
        _bind_stream(ctx, True)
        rc = _lib.load().fd_nn_descriptors(
            ctx.ptr, ctypes.c_void_p(m.data_ptr()), 1, layout, b, ch, h, w, ctypes.c_void_p(xy_t.data_ptr()),
            ctypes.c_void_p(cnt_t.data_ptr()) if cnt_t is not None else None, s, ctypes.c_void_p(res.data_ptr()), 1)
        _lib.check(ctx.ptr, rc)
        return res
    m = np.ascontiguousarray(desc_map, np.float32)
    b, ch, h, w = m.shape
    xy_h = np.ascontiguousarray(np.asarray(xy, np.float32).reshape(b, -1, 2))
    s = xy_h.shape[1]
    cnt_h = None if counts is None else np.ascontiguousarray(np.asarray(counts, np.int32).reshape(b))
    res = np.zeros((b, s, ch), np.float32)
    _bind_stream(ctx, False)
    rc = _lib.load().fd_nn_descriptors(
        ctx.ptr, ctypes.c_void_p(m.ctypes.data), 0, 0, b, ch, h, w, ctypes.c_void_p(xy_h.ctypes.data),
        ctypes.c_void_p(cnt_h.ctypes.data) if cnt_h is not None else None, s, ctypes.c_void_p(res.ctypes.data), 0)
    _lib.check(ctx.ptr, rc)
    return res


def build_net(seed: int = 0, head_gain: float = 100.0):
    """SuperPoint (DeTone et al. 2018): shared VGG encoder (1/8 resolution, 128 channels), detector
    head (65-way cell softmax -> full-resolution heatmap) and descriptor head (256-d, L2-normalised).
    Seeded random weights (the trained model is not available offline). With default init the
    65-way softmax is nearly uniform (every value ~1/65 < kMinResponse), so the detector head's
    logits are scaled by head_gain: at 100, ~5 % of a noise frame's pixels exceed 0.1 (a few
    thousand candidates per 640x480 frame), so that selection does the work a trained model gives it."""
    import torch
    from torch import nn

    class SuperPointNet(nn.Module):
        def __init__(self):
            super().__init__()
            c1, c2, c3, c4, c5, d1 = 64, 64, 128, 128, 256, 256
            self.pool = nn.MaxPool2d(2, 2)
            self.relu = nn.ReLU(inplace=True)
            self.conv1a = nn.Conv2d(1, c1, 3, 1, 1)
            self.conv1b = nn.Conv2d(c1, c1, 3, 1, 1)
            self.conv2a = nn.Conv2d(c1, c2, 3, 1, 1)
            self.conv2b = nn.Conv2d(c2, c2, 3, 1, 1)
            self.conv3a = nn.Conv2d(c2, c3, 3, 1, 1)
            self.conv3b = nn.Conv2d(c3, c3, 3, 1, 1)
            self.conv4a = nn.Conv2d(c3, c4, 3, 1, 1)
            self.conv4b = nn.Conv2d(c4, c4, 3, 1, 1)
            self.convPa = nn.Conv2d(c4, c5, 3, 1, 1)
            self.convPb = nn.Conv2d(c5, 65, 1, 1, 0)
            self.convDa = nn.Conv2d(c4, c5, 3, 1, 1)
            self.convDb = nn.Conv2d(c5, d1, 1, 1, 0)

        def forward(self, x):
            """x: [B, 1, H, W] in [0, 1] -> (heatmap [B, H, W] f32, descriptors [B, 256, H/8, W/8] f32)."""
            r = self.relu
            x = r(self.conv1b(r(self.conv1a(x))))
            x = self.pool(x)
            x = r(self.conv2b(r(self.conv2a(x))))
            x = self.pool(x)
            x = r(self.conv3b(r(self.conv3a(x))))
            x = self.pool(x)
            x = r(self.conv4b(r(self.conv4a(x))))
            semi = self.convPb(r(self.convPa(x))).float()
            prob = torch.softmax(semi, dim=1)[:, :-1]
            heat = torch.nn.functional.pixel_shuffle(prob, 8)[:, 0]
            desc = self.convDb(r(self.convDa(x))).float()
            desc = desc / desc.norm(dim=1, keepdim=True).clamp_min(1e-12)
            return heat, desc

    torch.manual_seed(seed)
    net = SuperPointNet()
    with torch.no_grad():
        net.convPb.weight.mul_(head_gain)
        net.convPb.bias.mul_(head_gain)
    return net


class SuperPointDetector:
    """NNFeaturePointDetector for the SuperPoint heatmap model, batched, on one GPU."""

    def __init__(self, options: Options | None = None, device: int = 0, dtype: str = "fp16", seed: int = 0):
        self._options = options or Options()
        self.device = device
        self.dtype = dtype
        self.seed = seed
        self.net = None

    def options(self) -> Options:
        return self._options

    def Initialize(self) -> bool:
        """nn_feature_point_detector.cpp:10-57: build the network, run it once on an all-ones image."""
        import torch

        if self._options.kModelType != "kSuperpointHeatmap":
            raise NotImplementedError("only kSuperpointHeatmap is provided (see module docstring)")
        dev = torch.device("cuda", self.device)
        net = build_net(self.seed).to(dev).eval()
        if self.dtype == "fp16":
            net = net.half()
        self.net = net.to(memory_format=torch.channels_last)
        # MIOpen solver choice (measured with tools/sp_find_probe.py, 64x640x480 fp16): exhaustive find
        # (benchmark=True) picks solvers worth 14.3 ms per 64 frames against 17.1 ms for immediate mode
        # (FD_SP_FIND_EXHAUSTIVE=0), but its first use also times the naive direct solver on every
        # conv shape (~30 s). That solver never wins, so it is left out of the search unless the caller
        # set the variable: first find ~10 s, ~0.6 s once MIOpen's user find-db holds the shapes.
        os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
        torch.backends.cudnn.benchmark = os.environ.get("FD_SP_FIND_EXHAUSTIVE", "1") == "1"
        ones = torch.ones((1, self._options.kMaxImageRows, self._options.kMaxImageCols), dtype=torch.uint8, device=dev)
        self.InferenceSession(ones)
        return True

    def InferenceSession(self, frames):
        """frames: u8 [B, H, W] device tensor -> (heatmap f32 [B, H, W], descriptors f32 [B, 256, H/8, W/8])."""
        import torch

        x = frames.unsqueeze(1).to(torch.float16 if self.dtype == "fp16" else torch.float32) / 255.0
        x = x.contiguous(memory_format=torch.channels_last)
        with torch.inference_mode():
            return self.net(x)

    def DetectGoodFeaturesWithDescriptor(self, frames, prior=None):
        """nn_feature_point_detector_superpoint.cpp:8-77 for a batch of device frames [B, H, W] (H, W
        multiples of 8). Returns (xy [B, S, 2], counts [B], descriptors [B, S, 256]) on the device:
        the new features of each frame and, when kComputeDescriptors, their descriptors (the
        reference also describes the priors: pass them through nn_descriptors)."""
        if self.net is None:
            raise RuntimeError("Initialize() first")
        heat, desc = self.InferenceSession(frames)
        xy, cnt = nn_select(heat, self._options, prior)
        d = nn_descriptors(desc, xy, cnt) if self._options.kComputeDescriptors else None
        return xy, cnt, d
