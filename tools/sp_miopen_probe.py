"""Probe: MIOpen's fused convolution + bias + ReLU (torch.miopen_convolution_relu) for the SuperPoint
encoder vs the current path (bias-free conv + fd_nn_bias_relu). Times the network forward on 64 frames
(640x480 fp16 channels-last) both ways and per layer, and the fused forward's difference to the module
forward. usage: python3 tools/sp_miopen_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from feature_detector_amd import superpoint as sp  # noqa: E402

dev = "cuda"
net = sp.build_net(0).half().to(dev).to(memory_format=torch.channels_last).eval()
g = torch.Generator(device=dev)
g.manual_seed(3)
x = torch.rand((64, 1, 480, 640), generator=g, device=dev).half().contiguous(memory_format=torch.channels_last)


def timeit(fn, n=10):
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def fused_cbr(conv, x, pool=False):
    y = torch.miopen_convolution_relu(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)
    return torch.nn.functional.max_pool2d(y, 2, 2) if pool else y


def forward_fused(x):
    x = fused_cbr(net.conv1b, fused_cbr(net.conv1a, x), pool=True)
    x = fused_cbr(net.conv2b, fused_cbr(net.conv2a, x), pool=True)
    x = fused_cbr(net.conv3b, fused_cbr(net.conv3a, x), pool=True)
    x = fused_cbr(net.conv4b, fused_cbr(net.conv4a, x))
    semi = net.convPb(fused_cbr(net.convPa, x)).float()
    desc = net.convDb(fused_cbr(net.convDa, x)).float()
    return semi, desc


def forward_cur(x):
    x = net.cbr(net.conv1b, net.cbr(net.conv1a, x), pool=True)
    x = net.cbr(net.conv2b, net.cbr(net.conv2a, x), pool=True)
    x = net.cbr(net.conv3b, net.cbr(net.conv3a, x), pool=True)
    x = net.cbr(net.conv4b, net.cbr(net.conv4a, x))
    semi = net.convPb(net.cbr(net.convPa, x)).float()
    desc = net.convDb(net.cbr(net.convDa, x)).float()
    return semi, desc


with torch.no_grad():
    a = forward_cur(x)
    try:
        b = forward_fused(x)
    except Exception as e:  # (MIOpen without the fusion for these shapes)
        print("fused forward failed:", e)
        sys.exit(0)
    for name, u, v in (("semi", a[0], b[0]), ("desc", a[1], b[1])):
        d = (u - v).abs().max().item()
        print(f"{name}: max |current - fused| = {d:.4g} (max |current| {u.abs().max().item():.4g})")
print(f"network (encoder + heads, no softmax): current {timeit(lambda: forward_cur(x)):.3f} ms, "
      f"fused {timeit(lambda: forward_fused(x)):.3f} ms per 64 frames")
# per layer
h = x
with torch.no_grad():
    for name, pool in (("conv1a", False), ("conv1b", True), ("conv2a", False), ("conv2b", True), ("conv3a", False),
                       ("conv3b", True), ("conv4a", False), ("conv4b", False)):
        conv = getattr(net, name)
        tc = timeit(lambda: net.cbr(conv, h, pool))
        tf = timeit(lambda: fused_cbr(conv, h, pool))
        tconv = timeit(lambda: torch.nn.functional.conv2d(h, conv.weight, None, conv.stride, conv.padding))
        print(f"{name} in {tuple(h.shape)}: current {tc:.3f} ms (conv alone {tconv:.3f}), fused {tf:.3f} ms")
        h = net.cbr(conv, h, pool)
