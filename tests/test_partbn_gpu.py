"""BatchNorm backward partials from the data-gradient epilogue of every conv kernel family
(round 6, ops.PartBN): a BatchNorm(+ReLU) layer without residual whose stored output feeds
exactly one conv -- the Bottleneck's bn2 -> conv3 1x1 (enc_hrnet.py:84-101), the 144-channel
branch's BasicBlock bn1 -> conv2 (:46-55), the inner units of a fuse down-chain (:199-218) --
gets (sum g, sum g*xhat) from that conv's data-gradient kernel (the persistent 1x1 GEMM or the
gather kernel, stride-2 parity classes included) instead of its own reduce pass.

Kernel level: dx equals vae2_conv2d_bwd_data bit for bit and the partial rows sum (in double)
to the fp64 reduction of the same terms.  Block / module level: PartBN on vs off (ops.PART_BN)
gives bit-identical forward outputs and running statistics and gradients within summation-
order noise."""
import ctypes

import pytest
import torch
import torch.nn as nn

from helpers import rel, rel_nz

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("case", [
    # (n, h, w of dx, dx channels = the BN layer's, dy channels, k, stride, relu)
    (2, 128, 256, 64, 256, 1, 1, True),   # Bottleneck conv3: persistent 1x1 GEMM dgrad
    (2, 32, 64, 72, 36, 1, 1, True),      # small 1x1: gather kernel
    (4, 16, 32, 144, 144, 3, 1, True),    # 144-channel branch conv2: gather, K split
    (2, 64, 128, 18, 36, 3, 2, True),     # stride 2: 4 parity classes, 16 + 2 remainder
    (3, 33, 47, 36, 72, 3, 2, False),     # odd sizes, no ReLU
    (2, 64, 128, 18, 18, 3, 2, True),     # fuse down-chain inner unit 18 -> 18 s2
])
def test_bnpart_every_kernel_family(case):
    from vae2 import _lib, ops
    from vae2._lib import call
    lib = _lib.load()
    n, h, w, c, co, k, st, relu = case
    pad = k // 2
    oh, ow = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    torch.manual_seed(7)
    x = ops.new_act((n, h, w, c), torch.empty(1, device=DEV))   # the BN layer's pre-BN r
    dy = ops.new_act((n, oh, ow, co), x)                         # gradient of the conv output
    with torch.no_grad():
        x.normal_(0.2, 1.3)
        dy.normal_()
    mean = x.reshape(-1, c).mean(0)
    invstd = 1.0 / (x.reshape(-1, c).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = torch.randn(c, device=DEV) * 0.5 + 1.0
    beta = torch.randn(c, device=DEV) * 0.5
    save = torch.cat([mean, invstd, gamma * invstd, beta - mean * gamma * invstd]).contiguous()
    wt = torch.randn(co, c, k, k, device=DEV) * 0.1
    wp1 = ops.packed_weight(wt, 1)
    xp, xd = ops.act_of(x)
    dyp, dyd = ops.act_of(dy)
    s = ops.stream_ptr()
    dx1, dx2 = ops.new_act((n, h, w, c), x), ops.new_act((n, h, w, c), x)
    dxd = ops.act_of(dx1)[1]
    call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dyd), ops.ptr(wp1), ops.ptr(dx1),
         ctypes.byref(dxd), k, st, pad, 0.0, s)
    rows = lib.vae2_conv2d_bwd_data_bnpart_rows(dyp, ctypes.byref(dyd), ctypes.byref(dxd), k,
                                                st, pad)
    assert rows > 0
    part = torch.full((2 * rows * c,), float("nan"), device=DEV)  # every row must be written
    call("vae2_conv2d_bwd_data_bnpart", dyp, ctypes.byref(dyd), ops.ptr(wp1), ops.ptr(dx2),
         ctypes.byref(dxd), k, st, pad, xp, ctypes.byref(xd), ops.ptr(save), int(relu),
         ops.ptr(part), s)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx2)
    got = part.view(2, rows, c).double().sum(1)
    assert bool(torch.isfinite(got).all())
    g = dx1.double().reshape(-1, c)
    xx = x.double().reshape(-1, c)
    if relu:
        mask = (xx * save[2 * c:3 * c].double() + save[3 * c:].double()) > 0
        g = torch.where(mask, g, torch.zeros_like(g))
    exact = torch.stack([g.sum(0), (g * (xx - mean.double()) * invstd.double()).sum(0)])
    assert rel(got, exact) < 1e-5, rel(got, exact)


def _counting(monkeypatch):
    from vae2 import ops
    made = []
    real = ops.PartBN

    class Counting(real):
        __slots__ = ()

        def __init__(self):
            super().__init__()
            made.append(self)

    monkeypatch.setattr(ops, "PartBN", Counting)
    return made


def _init(mod, g):
    with torch.no_grad():
        for m in mod.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) / m.weight[0].numel() ** 0.5)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.copy_(1.0 + 0.3 * torch.randn(m.weight.shape, generator=g))
                m.bias.copy_(0.3 * torch.randn(m.bias.shape, generator=g))


def _layer1_run(on, monkeypatch, seed=3):
    """layer1 (two Bottlenecks, the first with the downsample shortcut) at 128x256, B=2."""
    from vae2 import hrnet, ops
    monkeypatch.setattr(ops, "PART_BN", on)
    made = _counting(monkeypatch)
    torch.manual_seed(seed)
    blk = hrnet.make_layer(hrnet.Bottleneck, 64, 64, 2).to(DEV)
    _init(blk, torch.Generator().manual_seed(seed))
    x = ops.new_act((2, 128, 256, 64), torch.empty(1, device=DEV))
    with torch.no_grad():
        x.copy_(torch.randn(x.shape, generator=torch.Generator().manual_seed(seed + 1)).to(DEV))
    x.requires_grad_(True)
    y = hrnet.run_seq(blk, x)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(seed + 2)).to(DEV)
    torch.autograd.backward([y], [gy])
    torch.cuda.synchronize()
    return blk, [x], [y], made


def _stage4_run(on, monkeypatch, seed=4):
    """A W18 stage-4 HighResolutionModule (the 144-channel branch's conv2 is a gather-kernel
    conv; fuse rows with 2- and 3-unit down chains) at 32x64, B=2."""
    from helpers import build, make_cfg
    from vae2 import ops
    monkeypatch.setattr(ops, "PART_BN", on)
    made = _counting(monkeypatch)
    ed, _ = build(make_cfg(arch="w18", hw=(32, 64)))
    mod = ed.stage4[0].to(DEV)
    g = torch.Generator().manual_seed(seed)
    _init(mod, g)
    xs = []
    for c, h, w in [(18, 32, 64), (36, 16, 32), (72, 8, 16), (144, 4, 8)]:
        x = ops.new_act((2, h, w, c), torch.empty(1, device=DEV))
        with torch.no_grad():
            x.copy_(torch.randn(x.shape, generator=g).to(DEV))
        xs.append(x.requires_grad_(True))
    ys = mod.run(xs)
    gs = [torch.randn(y.shape, generator=g).to(DEV) for y in ys]
    torch.autograd.backward(ys, gs)
    torch.cuda.synchronize()
    return mod, xs, ys, made


@pytest.mark.parametrize("runner", ["layer1", "stage4"])
def test_partbn_equals_own_reduce_pass(runner, monkeypatch):
    run = _layer1_run if runner == "layer1" else _stage4_run
    ma, xa, ya, made_a = run(True, monkeypatch)
    mb, xb, yb, made_b = run(False, monkeypatch)
    # the partials path ran (its markers were armed with the pre-BN tensor), and the A/B
    # switch turns it off
    assert sum(1 for p in made_a if p.rows > 0) >= 2 and not made_b
    for u, v in zip(ya, yb):
        assert torch.equal(u, v)  # the forward is untouched
    for u, v in zip(xa, xb):
        assert rel_nz(u.grad, v.grad) < 1e-5
    for (n, p), (_, q) in zip(ma.named_parameters(), mb.named_parameters()):
        assert rel_nz(p.grad, q.grad) < 1e-5, n
    for (n, a), (_, b) in zip(ma.named_buffers(), mb.named_buffers()):
        if "running" in n:
            assert torch.equal(a, b), n
