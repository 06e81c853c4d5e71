"""The narrow-channel 3x3 weight-gradient kernel (csrc/wgrad_narrow.hip: 18 / 36 / 72
channels, columns ordered (dw, dh, ci)) against fp64 CPU references of the same
weight gradient (torch.nn.grad.conv2d_weight), with and without the input BatchNorm
(LazyBN: dW of conv(relu(bn(r))) from r), partial row / column tiles, channel slices
of wider NHWC buffers, and against the general direct kernel (tune key 7 = 0)."""
import ctypes

import pytest
import torch
from torch.nn.grad import conv2d_weight

from helpers import rel

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [
    # N, H, W, C (cin == cout), extra pixel-stride channels
    (8, 128, 256, 18, 0),   # the bench's 18-channel branch
    (8, 64, 128, 36, 0),    # 36-channel branch
    (8, 32, 64, 72, 0),     # 72 = 2 co slabs x 2 ci slabs
    (2, 13, 37, 18, 0),     # partial row and column tiles
    (3, 9, 70, 36, 4),      # partial tiles, wider pixel stride
    (1, 6, 40, 72, 8),
    (2, 4, 16, 18, 2),      # image narrower than a tile
]


def _run(x, dy, k7, save=None, relu=0, acc=False, dw0=None):
    """vae2_conv2d_bwd_weight(_bnin) with tune key 7 = k7; returns (dW, kernel names)."""
    from test_bench_instances_gpu import Recorder
    from vae2 import _lib, ops
    lib = _lib.load()
    cout, cin = dy.shape[3], x.shape[3]
    dw = dw0.clone() if dw0 is not None else torch.zeros(cout, cin, 3, 3, device=DEV)
    xp, xa = ops.act_of(x)
    dyp, dya = ops.act_of(dy)
    prev = lib.vae2_conv2d_set_tune(7, k7)
    try:
        size = lib.vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xa), ctypes.byref(dya), 3)
        ws = torch.empty(max(size, 1), device=DEV)
        with Recorder() as rec:
            if save is None:
                ops.call("vae2_conv2d_bwd_weight", xp, ctypes.byref(xa), dyp, ctypes.byref(dya),
                         ops.ptr(dw), None, 3, 1, 1, int(acc), ops.ptr(ws), size, ops.stream_ptr())
            else:
                ops.call("vae2_conv2d_bwd_weight_bnin", xp, ctypes.byref(xa), ops.ptr(save), relu,
                         dyp, ctypes.byref(dya), ops.ptr(dw), None, 3, 1, 1, int(acc),
                         ops.ptr(ws), size, ops.stream_ptr())
            torch.cuda.synchronize()
    finally:
        lib.vae2_conv2d_set_tune(7, prev)
    return dw, [k for _, _, ks in rec.calls for k in ks]


def _act(n, h, w, c, extra, g):
    from vae2 import ops
    t = torch.randn(n, h, w, c, generator=g)
    if extra:  # a channel slice of a wider buffer (pixel stride c + extra, 16-byte aligned)
        big = torch.zeros(n, h, w, c + extra, device=DEV)
        big[..., :c] = t.to(DEV)
        return big[..., :c], t
    a = ops.new_act((n, h, w, c), torch.empty(1, device=DEV))
    a.copy_(t.to(DEV))
    return a, t


@pytest.mark.parametrize("shape", SHAPES)
def test_wgrad_narrow_matches_fp64(shape):
    n, h, w, c, extra = shape
    g = torch.Generator().manual_seed(11 + c + h)
    x, xc = _act(n, h, w, c, extra, g)
    dy, dyc = _act(n, h, w, c, extra, g)
    dw, names = _run(x, dy, 1)
    assert any(k.startswith("wgrad3n_kernel") for k in names), names
    ref = conv2d_weight(xc.permute(0, 3, 1, 2).double(), (c, c, 3, 3),
                        dyc.permute(0, 3, 1, 2).double(), 1, 1)
    # fp32 sums over n*h*w pixels in another order than fp64: the direct kernel's bound
    assert rel(dw, ref) < 2e-6 * (1 + (n * h * w) ** 0.5 / 64), rel(dw, ref)
    dw_old, names_old = _run(x, dy, 0)
    assert not any(k.startswith("wgrad3n_kernel") for k in names_old), names_old
    assert rel(dw, dw_old) < 1e-5
    # the register-prefetch form (tune key 7 = 2): the same per-tile sums; its occupancy
    # (140 vs 112 VGPRs for 18 channels) can give another split plan, i.e. another order of
    # the partial-slab sum
    dw_pf, _ = _run(x, dy, 2)
    assert rel(dw_pf, dw) < 1e-5
    # the 8-wave form (key 7 = 3: the extra waves split the pixel chunks, summed through
    # LDS in wave order): the same sums in another order
    dw_8, names_8 = _run(x, dy, 3)
    assert any(k.startswith("wgrad3n_kernel") and k.endswith(", 8>") for k in names_8), names_8
    assert rel(dw_8, dw) < 1e-5


@pytest.mark.parametrize("shape", [(8, 128, 256, 18, 0), (2, 13, 37, 36, 4), (1, 6, 40, 72, 0)])
@pytest.mark.parametrize("relu", [0, 1])
def test_wgrad_narrow_input_bn(shape, relu):
    """LazyBN: dW of conv(relu?(r * scale + shift)) from r (in-image pixels only; the zero
    padding stays zero), accumulated onto an existing dW."""
    n, h, w, c, extra = shape
    g = torch.Generator().manual_seed(5 + c)
    x, xc = _act(n, h, w, c, extra, g)
    dy, dyc = _act(n, h, w, c, extra, g)
    mean, invstd = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.5
    gamma, beta = torch.randn(c, generator=g), torch.randn(c, generator=g)
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    save = torch.cat([mean, invstd, scale, shift]).to(DEV)
    dw0 = torch.randn(c, c, 3, 3, device=DEV)
    dw, names = _run(x, dy, 1, save=save, relu=relu, acc=True, dw0=dw0)
    assert any(k.startswith("wgrad3n_kernel") for k in names), names
    z = torch.addcmul(shift.double().view(1, 1, 1, c), xc.double(), scale.double().view(1, 1, 1, c))
    if relu:
        z = z.clamp_min(0)
    ref = conv2d_weight(z.permute(0, 3, 1, 2), (c, c, 3, 3), dyc.permute(0, 3, 1, 2).double(),
                        1, 1) + dw0.double().cpu()
    assert rel(dw, ref) < 2e-6 * (1 + (n * h * w) ** 0.5 / 64), rel(dw, ref)
