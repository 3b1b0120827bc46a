"""NN keypoints + descriptors: the networks in PyTorch-ROCm, the post-processing in
the HIP kernels behind fd_nn_select / fd_nn_select_list / fd_nn_descriptors.

Mirrors feature_detector::NNFeaturePointDetector (src/nn_feature_point_detector/
nn_feature_point_detector.h:12-86) for its four model types (ModelType, :15-20):
  Initialize()                          nn_feature_point_detector.cpp:10-57 (network + one warm-up run)
  DetectGoodFeaturesWithDescriptor()    nn_feature_point_detector_superpoint.cpp:8-112 / _disk.cpp:8-112
    InferenceSession                    -> the network (fp16 convs through MIOpen, fp32 outputs); DISK
                                           models take the gray frame as RGB (:96-99)
    heatmap models (kSuperpointHeatmap, kDiskHeatmap):
      CreateMask + candidates + selection -> fd_nn_select (GPU, std::multimap order)
      ExtractDescriptorsForSelectedFeatures -> fd_nn_descriptors for the priors and the new features
                                           (the reference describes every entry of all_pixel_uv)
    keypoint-list models (kSuperpointNms, kDiskNms: NMS in the graph):
      ArgSort + DirectlySelectGoodFeaturesWithDescriptors -> fd_nn_select_list (GPU selection +
                                           descriptor-row gather; new features only, as :223-227)

The reference loads trained ONNX models (onnx_models/*.onnx) that are not available here
(.MISSING_LARGE_BLOBS), and ONNX Runtime is absent: the networks are the published SuperPoint
architecture and a DISK-shaped U-Net with seeded random weights, with in-graph NMS + top-K heads for
the list models, so keypoints from them are meaningful for throughput only. The post-processing is
bit-exact to the oracle's restatement on any given network output.
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


def _prior_arrays(prior, b):
    """Per-frame prior features (list of (n_i, 2) (x, y) arrays) -> (flat float32 [sum, 2], counts int32)."""
    if prior is None:
        return None, None
    if len(prior) != b:
        raise ValueError("prior must have one entry per frame")
    pcnt = np.array([len(p) for p in prior], np.int32)
    pflat = (np.ascontiguousarray(np.concatenate([np.asarray(p, np.float32).reshape(-1, 2) for p in prior]))
             if pcnt.sum() > 0 else np.zeros((1, 2), np.float32))
    return pflat, pcnt


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
    pflat, pcnt = _prior_arrays(prior, b)
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


def nn_select_list(keypoints, scores, rows: int, cols: int, counts=None, options: Options | None = None, prior=None,
                   descriptors=None, out=None, ctx: Context | None = None):
    """fd_nn_select_list: the keypoint-list models' selection (DirectlySelectGoodFeaturesWithDescriptors).

    keypoints [B, K, 2] int64 (u, v) in a rows x cols frame, scores [B, K] float32, counts [B] int64
    (None: K each),
    descriptors [B, K, D] float32 or None. numpy inputs give numpy outputs; torch device tensors give
    device outputs (current stream). Returns (xy [B, max+1, 2], counts [B] int32, desc [B, max+1, D] or
    None): the new features per frame in selection order and their descriptor rows.
    prior: None or a list (per frame) of (n_i, 2) float arrays of (x, y), host memory.
    """
    o = options or Options()
    on_dev = _is_torch_device_tensor(scores)
    ctx = _resolve_ctx(ctx, scores)
    opts = _opts(o, float("inf"))
    stride = max(int(o.kMaxNumberOfDetectedFeatures), 1) + 1
    pflat, pcnt = _prior_arrays(prior, int(scores.shape[0]))
    if on_dev:
        import torch

        kp = keypoints.to(torch.int64).contiguous()
        sc = scores.to(torch.float32).contiguous()
        b, k = (int(v) for v in sc.shape)
        cnt_in = (torch.full((b,), k, dtype=torch.int64, device=sc.device) if counts is None
                  else counts.to(torch.int64).contiguous())
        dd = None if descriptors is None else descriptors.to(torch.float32).contiguous()
        dim = 0 if dd is None else int(dd.shape[2])
        if out is None:
            out = (torch.empty((b, stride, 2), dtype=torch.float32, device=sc.device),
                   torch.empty((b,), dtype=torch.int32, device=sc.device),
                   None if dd is None else torch.zeros((b, stride, dim), dtype=torch.float32, device=sc.device))
        xy, cnt, dout = out
        stride = xy.shape[1]
        ptrs = (kp.data_ptr(), sc.data_ptr(), cnt_in.data_ptr(), 0 if dd is None else dd.data_ptr(),
                0 if dout is None else dout.data_ptr(), xy.data_ptr(), cnt.data_ptr())
    else:
        kp = np.ascontiguousarray(keypoints, np.int64)
        sc = np.ascontiguousarray(scores, np.float32)
        b, k = sc.shape
        cnt_in = np.full((b,), k, np.int64) if counts is None else np.ascontiguousarray(counts, np.int64)
        dd = None if descriptors is None else np.ascontiguousarray(descriptors, np.float32)
        dim = 0 if dd is None else dd.shape[2]
        xy = np.zeros((b, stride, 2), np.float32)
        cnt = np.zeros((b,), np.int32)
        dout = None if dd is None else np.zeros((b, stride, dim), np.float32)
        ptrs = (kp.ctypes.data, sc.ctypes.data, cnt_in.ctypes.data, 0 if dd is None else dd.ctypes.data,
                0 if dout is None else dout.ctypes.data, xy.ctypes.data, cnt.ctypes.data)
    if tuple(kp.shape) != (b, k, 2):
        raise ValueError("keypoints must be [B, K, 2] matching scores [B, K]")
    _bind_stream(ctx, on_dev)
    vp = [ctypes.c_void_p(p) if p else None for p in ptrs]
    rc = _lib.load().fd_nn_select_list(
        ctx.ptr, vp[0], vp[1], vp[2], int(k), 1 if on_dev else 0, b, int(rows), int(cols), ctypes.byref(opts),
        ctypes.c_void_p(pflat.ctypes.data) if pflat is not None else None,
        ctypes.c_void_p(pcnt.ctypes.data) if pcnt is not None else None,
        vp[3], int(dim), vp[4], vp[5], int(stride), vp[6], 1 if on_dev else 0)
    _lib.check(ctx.ptr, rc)
    return xy, cnt, dout


def _ab_env(name: str, default=None):
    """A/B switch of the network's layer paths (FD_SP_*): read only with FD_DEBUG_AB set, so a stray
    variable in a user's environment does not change the code path."""
    if os.environ.get("FD_DEBUG_AB", "0") in ("", "0"):
        return default
    return os.environ.get(name, default)


def bias_relu(x, bias, pool: bool = False, out=None, ctx: Context | None = None):
    """fd_nn_bias_relu: relu(x + bias) (and the 2x2 max pool when pool) of a channels-last fp16
    activation [N, C, H, W] on the device, in one pass (torch's current stream). x is the output of a
    bias-free convolution; the result equals PyTorch's separate half-precision add / ReLU (/ MaxPool2d(2,
    2)) ops on it, bit for bit (not a conv-with-bias, whose bias is added before the rounding to half;
    and a NaN sum gives 0 here). out: preallocated result (may be x itself when not pooling)."""
    import torch

    if not (_is_torch_device_tensor(x) and x.dtype == torch.float16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("bias_relu: x must be a channels-last float16 [N, C, H, W] device tensor")
    n, c, h, w = x.shape
    if pool and (h % 2 or w % 2):
        raise ValueError("bias_relu: pooling needs even H and W")
    shape = (n, c, h // 2, w // 2) if pool else (n, c, h, w)
    if out is None:
        out = torch.empty(shape, dtype=torch.float16, device=x.device, memory_format=torch.channels_last)
    elif not (_is_torch_device_tensor(out) and out.device == x.device and out.dtype == torch.float16
              and tuple(out.shape) == shape and out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError(f"bias_relu: out must be a channels-last float16 {list(shape)} tensor on {x.device}")
    if bias.numel() != c:
        raise ValueError(f"bias_relu: bias has {bias.numel()} values for {c} channels")
    b = bias.detach().to(device=x.device, dtype=torch.float16).contiguous()
    ctx = _resolve_ctx(ctx, x)
    _bind_stream(ctx, True)
    rc = _lib.load().fd_nn_bias_relu(ctx.ptr, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                      int(b.numel()), ctypes.c_void_p(out.data_ptr()), int(n), int(h), int(w), int(c),
                                      1 if pool else 0)
    _lib.check(ctx.ptr, rc)
    return out


def heat_softmax(semi, bias=None, ctx: Context | None = None):
    """fd_nn_heat_softmax: SuperPoint's detector-head output from convPb's logits [N, 65, Hc, Wc]
    (channels-last fp16, on the device): softmax over the 65 channels in float, the dustbin dropped,
    pixel_shuffle(8) -> heat [N, 8 Hc, 8 Wc] float32, in one pass (PyTorch: float copy, softmax, slice,
    shuffle). bias (65 values): added to semi in half first (semi from a bias-free convolution). Within
    float rounding of torch.softmax((semi + bias).float(), 1)[:, :-1] shuffled."""
    import torch

    if not (_is_torch_device_tensor(semi) and semi.dtype == torch.float16 and semi.dim() == 4 and semi.shape[1] == 65
            and semi.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("heat_softmax: semi must be a channels-last float16 [N, 65, Hc, Wc] device tensor")
    n, _, hc, wc = semi.shape
    b = None
    if bias is not None:
        if bias.numel() != 65:
            raise ValueError("heat_softmax: bias must hold 65 values")
        b = bias.detach().to(device=semi.device, dtype=torch.float16).contiguous()
    heat = torch.empty((n, 8 * hc, 8 * wc), dtype=torch.float32, device=semi.device)
    ctx = _resolve_ctx(ctx, semi)
    _bind_stream(ctx, True)
    rc = _lib.load().fd_nn_heat_softmax(ctx.ptr, ctypes.c_void_p(semi.data_ptr()),
                                         ctypes.c_void_p(b.data_ptr() if b is not None else None),
                                         ctypes.c_void_p(heat.data_ptr()), int(n), int(hc), int(wc))
    _lib.check(ctx.ptr, rc)
    return heat


def desc_normalize(desc, bias=None, ctx: Context | None = None):
    """fd_nn_desc_normalize: SuperPoint's descriptor-head output from convDb's [N, C, Hc, Wc] (channels-last
    fp16, on the device): each cell's vector over its L2 norm (clamped to 1e-12) in float -> [N, C, Hc, Wc]
    float32 channels-last, in one pass (PyTorch: float copy, norm, division). bias (C values): added in
    half first (desc from a bias-free convolution). Within float rounding of d.float() /
    d.float().norm(dim=1, keepdim=True).clamp_min(1e-12), d = desc + bias."""
    import torch

    if not (_is_torch_device_tensor(desc) and desc.dtype == torch.float16 and desc.dim() == 4 and desc.shape[1] % 8 == 0
            and desc.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("desc_normalize: desc must be a channels-last float16 [N, C, Hc, Wc] device tensor, C % 8 == 0")
    n, c, hc, wc = desc.shape
    b = None
    if bias is not None:
        if bias.numel() != c:
            raise ValueError(f"desc_normalize: bias must hold {c} values")
        b = bias.detach().to(device=desc.device, dtype=torch.float16).contiguous()
    out = torch.empty((n, c, hc, wc), dtype=torch.float32, device=desc.device, memory_format=torch.channels_last)
    ctx = _resolve_ctx(ctx, desc)
    _bind_stream(ctx, True)
    rc = _lib.load().fd_nn_desc_normalize(ctx.ptr, ctypes.c_void_p(desc.data_ptr()),
                                           ctypes.c_void_p(b.data_ptr() if b is not None else None),
                                           ctypes.c_void_p(out.data_ptr()), int(n) * int(hc) * int(wc), int(c))
    _lib.check(ctx.ptr, rc)
    return out


def conv1_bias_relu(x, weight, bias, out=None, ctx: Context | None = None):
    """fd_nn_conv3x3_c1: the encoder's first layer (1 input channel, 3x3, stride 1, padding 1) with its bias
    and ReLU in one pass: x [N, 1, H, W] fp16 on the device -> [N, C, H, W] fp16 channels-last. The 9
    products are summed in float and rounded to half, then the bias is added in float and rounded (as the
    bias-free convolution followed by bias_relu); within fp16 rounding of PyTorch's convolution + ReLU."""
    import torch

    if not (x.is_cuda and x.dtype == torch.float16 and x.dim() == 4 and x.shape[1] == 1
            and (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last))):
        raise ValueError("conv1_bias_relu: x must be a [N, 1, H, W] float16 device tensor")
    n, _, h, w = x.shape
    c = weight.shape[0]
    if tuple(weight.shape) != (c, 1, 3, 3) or weight.dtype != torch.float16 or bias.numel() != c:
        raise ValueError("conv1_bias_relu: weight must be [C, 1, 3, 3] float16 and bias C values")
    if out is None:
        out = torch.empty((n, c, h, w), dtype=torch.float16, device=x.device, memory_format=torch.channels_last)
    elif not (out.dtype == torch.float16 and tuple(out.shape) == (n, c, h, w)
              and out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError(f"conv1_bias_relu: out must be a channels-last float16 {[n, c, h, w]} tensor")
    ctx = _resolve_ctx(ctx, x)
    _bind_stream(ctx, True)
    wt = weight.detach().to(device=x.device, dtype=torch.float16).contiguous()  # (the kernel reads it on x's device)
    b = bias.detach().to(device=x.device, dtype=torch.float16).contiguous()
    rc = _lib.load().fd_nn_conv3x3_c1(ctx.ptr, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wt.data_ptr()),
                                       ctypes.c_void_p(b.data_ptr()), c, ctypes.c_void_p(out.data_ptr()), n, h, w)
    _lib.check(ctx.ptr, rc)
    return out


def pack_conv3x3_weight(weight):
    """[C_out, C_in, 3, 3] -> [9 taps (ky, kx)][C_out][C_in] contiguous (fd_nn_conv3x3_c64's filter layout)."""
    return weight.detach().permute(2, 3, 0, 1).reshape(9, weight.shape[0], weight.shape[1]).contiguous()


def conv64_bias_relu(x, weight, bias, pool: bool = False, out=None, ctx: Context | None = None, packed=None):
    """fd_nn_conv3x3_c64: 3x3 convolution from 64 channels to a multiple of 64 (stride 1, padding 1) + bias +
    ReLU (+ 2x2 max pool) on the matrix cores, one call per 64-output-channel block: x [N, 64, H, W] fp16
    channels-last on the device -> [N, C_out, H(/2), W(/2)] fp16 channels-last. fp16 products summed in
    float, the sum rounded to half, then the bias added in float and rounded (as the bias-free
    convolution + bias_relu path). packed: the filter's blocks already in pack_conv3x3_weight's layout
    (a list, one per 64 output channels; reused across calls)."""
    import torch

    if not (x.is_cuda and x.dtype == torch.float16 and x.dim() == 4 and x.shape[1] == 64
            and x.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("conv64_bias_relu: x must be a channels-last float16 [N, 64, H, W] device tensor")
    n, c, h, w = x.shape
    co = weight.shape[0]
    if co % 64 or tuple(weight.shape) != (co, 64, 3, 3) or bias.numel() != co:
        raise ValueError("conv64_bias_relu: weight must be [64 k, 64, 3, 3] and bias as many values")
    if pool and (h % 2 or w % 2):
        raise ValueError("conv64_bias_relu: pooling needs even H and W")
    shape = (n, co, h // 2, w // 2) if pool else (n, co, h, w)
    if out is None:
        out = torch.empty(shape, dtype=torch.float16, device=x.device, memory_format=torch.channels_last)
    elif not (out.dtype == torch.float16 and tuple(out.shape) == shape
              and out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError(f"conv64_bias_relu: out must be a channels-last float16 {list(shape)} tensor")
    if packed is None:
        packed = [pack_conv3x3_weight(weight[k:k + 64].to(device=x.device, dtype=torch.float16)) for k in range(0, co, 64)]
    elif any(wp.device != x.device or wp.dtype != torch.float16 or tuple(wp.shape) != (9, 64, 64) for wp in packed) \
            or len(packed) != co // 64:
        raise ValueError(f"conv64_bias_relu: packed must be {co // 64} float16 [9, 64, 64] blocks on {x.device}")
    b = bias.detach().to(device=x.device, dtype=torch.float16).contiguous()
    ctx = _resolve_ctx(ctx, x)
    _bind_stream(ctx, True)
    for blk, wp in enumerate(packed):
        bb = b[blk * 64:(blk + 1) * 64]
        rc = _lib.load().fd_nn_conv3x3_c64(ctx.ptr, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wp.data_ptr()),
                                            ctypes.c_void_p(bb.data_ptr()), ctypes.c_void_p(out.data_ptr()), n, h, w,
                                            1 if pool else 0, co, blk * 64)
        _lib.check(ctx.ptr, rc)
    return out


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


MODEL_TYPES = ("kSuperpointHeatmap", "kSuperpointNms", "kDiskHeatmap", "kDiskNms")  # ModelType (:15-20)
DESCRIPTOR_DIM = {"superpoint": 256, "disk": 128}  # SuperpointDescriptorType / DiskDescriptorType


def simple_nms(heat, radius: int):
    """In-graph NMS of the keypoint-list models (the max-pool suppression SuperPoint/DISK exports use):
    a score survives where it is the maximum of its (2r+1)^2 window, twice refined around the kept ones."""
    import torch
    import torch.nn.functional as F

    def mp(x):
        return F.max_pool2d(x, kernel_size=2 * radius + 1, stride=1, padding=radius)

    x = heat[:, None]
    zeros = torch.zeros_like(x)
    keep = x == mp(x)
    for _ in range(2):
        supp = mp(keep.float()) > 0
        supp_x = torch.where(supp, zeros, x)
        keep = keep | ((supp_x == mp(supp_x)) & ~supp)
    return torch.where(keep, x, zeros)[:, 0]


def top_k_keypoints(heat, k: int):
    """heat [B, H, W] -> (keypoints [B, k, 2] int64 (u, v), scores [B, k] float32), best first."""
    import torch

    b, h, w = heat.shape
    sc, idx = heat.reshape(b, -1).topk(min(k, h * w), dim=1)
    kp = torch.stack([idx % w, idx // w], dim=2).to(torch.int64)
    return kp, sc.float()


def build_net(seed: int = 0, head_gain: float = 100.0, nms: bool = False, top_k: int = 1024):
    """SuperPoint (DeTone et al. 2018): shared VGG encoder (1/8 resolution, 128 channels), detector
    head (65-way cell softmax -> full-resolution heatmap) and descriptor head (256-d, L2-normalised).
    Seeded random weights (the trained model is not available offline). With default init the
    65-way softmax is nearly uniform (every value ~1/65 < kMinResponse), so the detector head's
    logits are scaled by head_gain: at 100, ~5 % of a noise frame's pixels exceed 0.1 (a few
    thousand candidates per 640x480 frame), so that selection does the work a trained model gives it.
    nms=True (kSuperpointNms): the heatmap goes through simple_nms (radius 4) and top_k keypoints are
    returned with their scores and bilinearly sampled, normalised descriptors."""
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

        def cbr(self, conv, x, pool=False):
            """conv -> ReLU (-> MaxPool2d(2, 2)): fp16 channels-last activations run the convolution
            without its bias and fd_nn_bias_relu for bias, ReLU and pooling in one pass (PyTorch would make
            three or four elementwise passes over the activation); other inputs take the torch modules."""
            if x.dtype == torch.float16 and x.is_cuda and conv.in_channels == 1 and conv.kernel_size == (3, 3) \
                    and conv.stride == (1, 1) and conv.padding == (1, 1) and conv.out_channels in (8, 16, 32, 64, 128, 256) \
                    and x.dim() == 4 and x.shape[1] == 1 and not pool and not _ab_env("FD_SP_UNFUSED") \
                    and not _ab_env("FD_SP_NO_CONV1"):  # (A/B switches)
                # first layer: write-bound (9 MACs per output), one pass instead of convolution + bias pass
                return conv1_bias_relu(x.contiguous(), conv.weight, conv.bias)
            if x.dtype == torch.float16 and x.is_cuda and conv.in_channels == 64 and conv.out_channels % 64 == 0 \
                    and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1) \
                    and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) \
                    and (not pool or (x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)) \
                    and not _ab_env("FD_SP_UNFUSED") and not _ab_env("FD_SP_NO_C64") \
                    and (conv.out_channels == 64 or not _ab_env("FD_SP_C64_ONLY64")):  # (A/B switches)
                # 64 -> 64 k layers on the matrix cores with bias, ReLU and pooling in the epilogue
                # one packed copy per layer, replaced when the weight changes (in-place update, reload, device)
                tag = (conv.weight.data_ptr(), conv.weight._version, x.device)
                cache = self.__dict__.setdefault("_fd_packed", {})
                hit = cache.get(id(conv))
                if hit is None or hit[0] != tag:
                    hit = (tag, [pack_conv3x3_weight(conv.weight[k:k + 64].to(device=x.device, dtype=torch.float16))
                                 for k in range(0, conv.out_channels, 64)])
                    cache[id(conv)] = hit
                return conv64_bias_relu(x, conv.weight, conv.bias, pool, packed=hit[1])
            if x.dtype == torch.float16 and x.is_cuda and x.is_contiguous(memory_format=torch.channels_last) \
                    and conv.out_channels % 8 == 0 and not _ab_env("FD_SP_UNFUSED"):  # (A/B switch)
                y = torch.nn.functional.conv2d(x, conv.weight, None, conv.stride, conv.padding)
                if y.is_contiguous(memory_format=torch.channels_last):
                    return bias_relu(y, conv.bias, pool, out=None if pool else y)
                x = y + conv.bias.view(1, -1, 1, 1)
                x = self.relu(x)
                return self.pool(x) if pool else x
            x = self.relu(conv(x))
            return self.pool(x) if pool else x

        @staticmethod
        def fused_heads(semi, desc):
            """The heads' output stages run as fd_nn_heat_softmax / fd_nn_desc_normalize when the logits are
            channels-last fp16 on the device (FD_SP_UNFUSED=1 or FD_SP_TORCH_HEADS=1: PyTorch's ops, A/B)."""
            return (semi.is_cuda and semi.dtype == torch.float16 and semi.shape[1] == 65
                    and semi.is_contiguous(memory_format=torch.channels_last)
                    and desc.is_cuda and desc.dtype == torch.float16 and desc.shape[1] % 8 == 0
                    and desc.is_contiguous(memory_format=torch.channels_last)
                    and not _ab_env("FD_SP_UNFUSED") and not _ab_env("FD_SP_TORCH_HEADS"))

        def first_layers(self, x):
            """conv1a -> ReLU -> conv1b -> ReLU -> MaxPool2d(2, 2), layer by layer through cbr (conv1a's
            write-bound pass, then conv1b on the matrix cores). conv1a recomputed inside conv1b's tiles (the
            full-resolution activation never written) measured slower in both K10 forms -- 4.75-4.78 vs
            4.68-4.79 ms per 64-frame forward in round 5, 4.19-4.38 vs 4.09-4.13 ms once conv1b kept two tiles
            in flight per CU (profiles/r05_sp_ab.txt, r06_sp_fused_ab.txt) -- and was removed."""
            return self.cbr(self.conv1b, self.cbr(self.conv1a, x), pool=True)

        def forward(self, x):
            """x: [B, 1, H, W] in [0, 1] -> (heatmap [B, H, W] f32, descriptors [B, 256, H/8, W/8] f32), or
            with nms (keypoints [B, K, 2] int64, scores [B, K] f32, descriptors [B, K, 256] f32)."""
            x = self.first_layers(x)
            x = self.cbr(self.conv2b, self.cbr(self.conv2a, x), pool=True)
            x = self.cbr(self.conv3b, self.cbr(self.conv3a, x), pool=True)
            x = self.cbr(self.conv4b, self.cbr(self.conv4a, x))
            xp, xd = self.cbr(self.convPa, x), self.cbr(self.convDa, x)
            semi = desc = None
            if xp.is_cuda and xp.dtype == torch.float16 and xd.dtype == torch.float16 \
                    and not _ab_env("FD_SP_UNFUSED") and not _ab_env("FD_SP_TORCH_HEADS"):  # (A/B switches)
                # bias-free head convolutions: their biases go into the output stages below
                semi = torch.nn.functional.conv2d(xp, self.convPb.weight, None, self.convPb.stride, self.convPb.padding)
                desc = torch.nn.functional.conv2d(xd, self.convDb.weight, None, self.convDb.stride, self.convDb.padding)
                if self.fused_heads(semi, desc):  # the heads' output stages in one pass each (fd_nn.hip)
                    heat, desc = heat_softmax(semi, self.convPb.bias), desc_normalize(desc, self.convDb.bias)
                    semi = None
                else:
                    semi = semi + self.convPb.bias.view(1, -1, 1, 1)
                    desc = desc + self.convDb.bias.view(1, -1, 1, 1)
            else:
                semi, desc = self.convPb(xp), self.convDb(xd)
            if semi is not None:
                prob = torch.softmax(semi.float(), dim=1)[:, :-1]
                heat = torch.nn.functional.pixel_shuffle(prob, 8)[:, 0]
                desc = desc.float()
                desc = desc / desc.norm(dim=1, keepdim=True).clamp_min(1e-12)
            if not nms:
                return heat, desc
            kp, sc = top_k_keypoints(simple_nms(heat, 4), top_k)
            h, w = heat.shape[1:]
            # descriptor at each keypoint: bilinear on the 1/8 map at the cell-centred position
            grid = torch.stack([(kp[..., 0].float() + 0.5) / w * 2 - 1, (kp[..., 1].float() + 0.5) / h * 2 - 1], -1)
            d = torch.nn.functional.grid_sample(desc, grid[:, None], mode="bilinear", align_corners=False)[:, :, 0]
            d = d / d.norm(dim=1, keepdim=True).clamp_min(1e-12)
            return kp, sc, d.transpose(1, 2).contiguous()

    torch.manual_seed(seed)
    net = SuperPointNet()
    with torch.no_grad():
        net.convPb.weight.mul_(head_gain)
        net.convPb.bias.mul_(head_gain)
    return net


def build_disk(seed: int = 0, nms: bool = False, top_k: int = 1024, head_gain: float = 8.0):
    """DISK-shaped network (Tyszkiewicz et al. 2020): a U-Net on the RGB frame whose full-resolution
    output holds 128 descriptor channels and one detection channel. Seeded random weights (the
    trained disk.onnx is not available); the detection logits are scaled by head_gain and pass a
    sigmoid, so a few percent of a noise frame's pixels exceed kMinResponse. nms=True (kDiskNms):
    simple_nms (radius 2) + top_k keypoints with the descriptor rows at their pixels."""
    import torch
    from torch import nn

    def block(ci, co):
        return nn.Sequential(nn.Conv2d(ci, co, 3, 1, 1), nn.ReLU(inplace=True), nn.Conv2d(co, co, 3, 1, 1),
                             nn.ReLU(inplace=True))

    class DiskNet(nn.Module):
        def __init__(self):
            super().__init__()
            ch = (32, 64, 64, 128)
            self.enc = nn.ModuleList([block(3, ch[0]), block(ch[0], ch[1]), block(ch[1], ch[2]), block(ch[2], ch[3])])
            self.up = nn.ModuleList([nn.ConvTranspose2d(ch[3], ch[2], 2, 2), nn.ConvTranspose2d(ch[2], ch[1], 2, 2),
                                     nn.ConvTranspose2d(ch[1], ch[0], 2, 2)])
            self.dec = nn.ModuleList([block(2 * ch[2], ch[2]), block(2 * ch[1], ch[1]), block(2 * ch[0], ch[0])])
            self.head = nn.Conv2d(ch[0], 129, 1)
            self.pool = nn.MaxPool2d(2, 2)

        def forward(self, x):
            """x: [B, 3, H, W] in [0, 1] -> (heatmap [B, H, W] f32, descriptors [B, 128, H, W] f32), or
            with nms (keypoints [B, K, 2] int64, scores [B, K] f32, descriptors [B, K, 128] f32)."""
            skips = []
            for i, e in enumerate(self.enc):
                x = e(x if i == 0 else self.pool(x))
                skips.append(x)
            for u, d, sk in zip(self.up, self.dec, reversed(skips[:-1])):
                x = d(torch.cat([u(x), sk], dim=1))
            out = self.head(x).float()
            heat = torch.sigmoid(out[:, 128] * head_gain)
            desc = out[:, :128]
            desc = desc / desc.norm(dim=1, keepdim=True).clamp_min(1e-12)
            if not nms:
                return heat, desc
            kp, sc = top_k_keypoints(simple_nms(heat, 2), top_k)
            b = torch.arange(desc.shape[0], device=desc.device)[:, None]
            d = desc.permute(0, 2, 3, 1)[b, kp[..., 1], kp[..., 0]]
            return kp, sc, d.contiguous()

    torch.manual_seed(seed)
    return DiskNet()


@dataclass
class NNResult:
    """DetectGoodFeaturesWithDescriptor's outputs for a batch: xy [B, S, 2] / counts [B] (the new
    features), descriptors [B, S, D] (their rows), prior_descriptors [B, P, D] (heatmap models: the
    reference's descriptors of the incoming features, all_pixel_uv[0..P), per frame counts as the
    priors given; None for the keypoint-list models, whose reference returns new rows only). Unpacks as
    (xy, counts, descriptors)."""
    xy: object
    counts: object
    descriptors: object
    prior_descriptors: object = None

    def __iter__(self):
        return iter((self.xy, self.counts, self.descriptors))


class NNFeaturePointDetector:
    """NNFeaturePointDetector (nn_feature_point_detector.h:12-86), batched, on one GPU."""

    def __init__(self, options: Options | None = None, device: int = 0, dtype: str = "fp16", seed: int = 0,
                 top_k: int = 1024):
        self._options = options or Options()
        self.device = device
        self.dtype = dtype
        self.seed = seed
        self.top_k = top_k
        self.net = None

    def options(self) -> Options:
        return self._options

    @property
    def is_disk(self) -> bool:
        return self._options.kModelType.startswith("kDisk")

    @property
    def is_list_model(self) -> bool:
        return self._options.kModelType.endswith("Nms")

    def Initialize(self) -> bool:
        """nn_feature_point_detector.cpp:10-57: build the model's network, run it once on an all-ones image."""
        import torch

        mt = self._options.kModelType
        if mt not in MODEL_TYPES:
            raise ValueError(f"unknown kModelType {mt!r} (one of {MODEL_TYPES})")
        dev = torch.device("cuda", self.device)
        net = (build_disk(self.seed, nms=self.is_list_model, top_k=self.top_k) if self.is_disk
               else build_net(self.seed, nms=self.is_list_model, top_k=self.top_k))
        net = net.to(dev).eval()
        if self.dtype == "fp16":
            net = net.half()
        self.net = net.to(memory_format=torch.channels_last)
        # MIOpen solver choice (measured with tools/sp_find_probe.py, 64x640x480 fp16): exhaustive find
        # (benchmark=True) picks solvers worth 14.3 ms per 64 frames against 17.1 ms for immediate mode
        # (FD_SP_FIND_EXHAUSTIVE=0), but its first use also times the naive direct solver on every
        # conv shape (~30 s). That solver never wins, so it is left out of the search unless the caller
        # set the variable: first find ~10 s, ~0.6 s once MIOpen's user find-db holds the shapes.
        os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
        torch.backends.cudnn.benchmark = _ab_env("FD_SP_FIND_EXHAUSTIVE", "1") == "1"
        ones = torch.ones((1, self._options.kMaxImageRows, self._options.kMaxImageCols), dtype=torch.uint8, device=dev)
        self.InferenceSession(ones)
        return True

    def InferenceSession(self, frames):
        """frames: u8 [B, H, W] device tensor (H, W multiples of 8) -> the network's outputs: heatmap
        models (heatmap f32 [B, H, W], descriptor map f32 [B, D, h, w]); list models (keypoints
        int64 [B, K, 2], scores f32 [B, K], descriptors f32 [B, K, D]). DISK models see the gray frame as
        RGB (OnnxRuntime::ConvertGrayImageToRgbTensor, nn_feature_point_detector.cpp:96-99)."""
        import torch

        x = frames.unsqueeze(1).to(torch.float16 if self.dtype == "fp16" else torch.float32) / 255.0
        if self.is_disk:
            x = x.expand(-1, 3, -1, -1)
        x = x.contiguous(memory_format=torch.channels_last)
        with torch.inference_mode():
            return self.net(x)

    def DetectGoodFeaturesWithDescriptor(self, frames, prior=None) -> NNResult:
        """nn_feature_point_detector_superpoint.cpp:8-112 / nn_feature_point_detector_disk.cpp:8-112 for a
        batch of device frames [B, H, W]. prior: None or a list (per frame) of (n_i, 2) (x, y) arrays
        (the incoming all_pixel_uv). Returns an NNResult on the device."""
        import torch

        if self.net is None:
            raise RuntimeError("Initialize() first")
        o = self._options
        out = self.InferenceSession(frames)
        if self.is_list_model:
            kp, sc, dl = out
            xy, cnt, d = nn_select_list(kp, sc, int(frames.shape[1]), int(frames.shape[2]), None, o, prior, dl)
            return NNResult(xy, cnt, d, None)
        heat, desc = out
        xy, cnt = nn_select(heat, o, prior)
        d = nn_descriptors(desc, xy, cnt)
        pd = None
        if prior is not None:  # ExtractDescriptorsForSelectedFeatures runs over all_pixel_uv (priors first)
            p = max(max((len(q) for q in prior), default=0), 1)
            pxy = np.zeros((len(prior), p, 2), np.float32)
            for i, q in enumerate(prior):
                q = np.asarray(q, np.float32).reshape(-1, 2)
                pxy[i, :len(q)] = q
            pcnt = torch.tensor([len(q) for q in prior], dtype=torch.int32, device=desc.device)
            pd = nn_descriptors(desc, torch.from_numpy(pxy).to(desc.device), pcnt)
        return NNResult(xy, cnt, d, pd)


SuperPointDetector = NNFeaturePointDetector  # (kSuperpointHeatmap by default)
