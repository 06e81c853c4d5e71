"""BatchNorm fused into the consumer conv (ops.LazyBN, ABI 9): BasicBlock's bn1 -> relu
-> conv2 with the normalised activation never stored (enc_hrnet.py:46-55).

The forward (conv2 normalising its input while staging it) and the weight gradient are
the same arithmetic as normalising first, so outputs match the stored path bit for bit;
the backward partials come from conv2's data-gradient epilogue instead of a separate
reduce pass, i.e. the same per-element terms summed in another order (fp32 rounding)."""
import ctypes

import pytest
import torch
import torch.nn as nn

from helpers import rel, rel_nz

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _blocks(seed, chans):
    from vae2 import hrnet
    torch.manual_seed(seed)
    blocks = [hrnet.BasicBlock(c, c).to(DEV) for c in chans]
    for b in blocks:  # away from the reference init's (gamma 1, beta 0) to exercise masks
        for bn in (b.bn1, b.bn2):
            nn.init.normal_(bn.weight, 1.0, 0.3)
            nn.init.normal_(bn.bias, 0.0, 0.3)
    return blocks


def _run(lazy, seed, chans, shapes, monkeypatch):
    from vae2 import hrnet, ops
    monkeypatch.setattr(ops, "LAZY_BN", lazy)
    monkeypatch.setattr(ops, "MASK_BYTES", lazy)  # bn2's ReLU mask as bytes vs y
    made = []
    real = ops.LazyBN

    class Counting(real):
        __slots__ = ()

        def __init__(self):
            super().__init__()
            made.append(self)

    monkeypatch.setattr(ops, "LazyBN", Counting)
    blocks = _blocks(seed, chans)
    torch.manual_seed(seed + 1)
    xs = []
    for (n, h, w), c in zip(shapes, chans):
        x = ops.new_act((n, h, w, c), torch.empty(1, device=DEV))
        with torch.no_grad():
            x.normal_()
        xs.append(x.requires_grad_(True))
    ys = hrnet.run_blocks_lockstep(blocks, xs)
    torch.manual_seed(seed + 2)
    gs = [torch.randn_like(y) for y in ys]
    torch.autograd.backward(ys, gs)
    torch.cuda.synchronize()
    return blocks, xs, ys, len(made)


@pytest.mark.parametrize("case", [
    # (chans, (n, h, w) per branch): W18 branch widths where the direct 3x3 kernels run
    # (>= 256 tiles: 18 with the VALU remainder, 36 / 72 on MFMA tiles); 144 at 4x8 takes
    # the gather kernel -> stored (a mixed level)
    ([18, 36, 72, 144], [(2, 128, 256), (8, 64, 128), (32, 32, 64), (2, 4, 8)]),
    # partial row / column tiles
    ([18, 36], [(3, 130, 200), (12, 65, 100)]),
])
def test_lazy_bn_block_equals_stored(case, monkeypatch):
    chans, shapes = case
    ba, xa, ya, na = _run(True, 11, chans, shapes, monkeypatch)
    bb, xb, yb, nb = _run(False, 11, chans, shapes, monkeypatch)
    assert na >= 1 and nb == 0  # the fused path ran (and the A/B switch turns it off)
    for u, v in zip(ya, yb):
        assert torch.equal(u, v)  # forward: bit-identical
    for u, v in zip(xa, xb):
        assert rel_nz(u.grad, v.grad) < 1e-5
    for p, q in zip(ba, bb):
        for m, k in ((p.conv1, q.conv1), (p.conv2, q.conv2)):
            assert rel_nz(m.weight.grad, k.weight.grad) < 1e-5
        for m, k in ((p.bn1, q.bn1), (p.bn2, q.bn2)):
            assert rel_nz(m.weight.grad, k.weight.grad) < 1e-5
            assert rel_nz(m.bias.grad, k.bias.grad) < 1e-5
            assert torch.equal(m.running_mean, k.running_mean)
            assert torch.equal(m.running_var, k.running_var)


def test_bnpart_partials_equal_bwd_reduce():
    """vae2_conv2d_bwd_data_bnpart: dx equals vae2_conv2d_bwd_data bit for bit, and its
    partial rows sum (in double) to vae2_bn_relu_bwd_reduce's within fp32 rounding;
    vae2_conv2d_fwd_bnin / vae2_conv2d_bwd_weight_bnin equal the stored path bit for bit."""
    from vae2 import _lib, ops
    from vae2._lib import call
    lib = _lib.load()
    torch.manual_seed(5)
    n, h, w, c = 8, 64, 128, 18
    x = ops.new_act((n, h, w, c), torch.empty(1, device=DEV))  # pre-BN tensor of bn1
    dy = ops.new_act((n, h, w, c), x)                           # gradient of conv2's output
    with torch.no_grad():
        x.normal_(0.3, 1.2)
        dy.normal_()
    mean = x.reshape(-1, c).mean(0)
    invstd = 1.0 / (x.reshape(-1, c).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = torch.randn(c, device=DEV) * 0.5 + 1.0
    beta = torch.randn(c, device=DEV) * 0.5
    save = torch.cat([mean, invstd, gamma * invstd, beta - mean * gamma * invstd]).contiguous()
    wt = torch.randn(c, c, 3, 3, device=DEV) * 0.1
    wp0, wp1 = ops.packed_weight(wt, 0), ops.packed_weight(wt, 1)
    xp, xd = ops.act_of(x)
    dyp, dyd = ops.act_of(dy)
    s = ops.stream_ptr()
    assert lib.vae2_conv2d_bnin_ok(xp, ctypes.byref(xd), ctypes.byref(dyd), 3, 1, 1)
    # stored path: z = relu(x*scale + shift)
    z = ops.new_act((n, h, w, c), x)
    zp, zd = ops.act_of(z)
    call("vae2_bn_apply", xp, ctypes.byref(xd), ops.ptr(save), None, ctypes.byref(xd), zp,
         ctypes.byref(zd), 1, s)
    y1, y2 = ops.new_act((n, h, w, c), x), ops.new_act((n, h, w, c), x)
    call("vae2_conv2d_fwd", zp, ctypes.byref(zd), ops.ptr(wp0), None, ops.ptr(y1),
         ctypes.byref(ops.act_of(y1)[1]), 3, 1, 1, 0.0, None, s)
    call("vae2_conv2d_fwd_bnin", xp, ctypes.byref(xd), ops.ptr(save), 1, ops.ptr(wp0), None,
         ops.ptr(y2), ctypes.byref(ops.act_of(y2)[1]), 3, 1, 1, 0.0, None, s)
    size = lib.vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xd), ctypes.byref(dyd), 3)
    ws = torch.empty(size, device=DEV)
    dw1, dw2 = torch.zeros_like(wt), torch.zeros_like(wt)
    call("vae2_conv2d_bwd_weight", zp, ctypes.byref(zd), dyp, ctypes.byref(dyd), ops.ptr(dw1),
         None, 3, 1, 1, 0, ops.ptr(ws), size, s)
    call("vae2_conv2d_bwd_weight_bnin", xp, ctypes.byref(xd), ops.ptr(save), 1, dyp,
         ctypes.byref(dyd), ops.ptr(dw2), None, 3, 1, 1, 0, ops.ptr(ws), size, s)
    # data gradient + the bn1 backward partials
    dx1, dx2 = ops.new_act((n, h, w, c), x), ops.new_act((n, h, w, c), x)
    dxd = ops.act_of(dx1)[1]
    call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dyd), ops.ptr(wp1), ops.ptr(dx1),
         ctypes.byref(dxd), 3, 1, 1, 0.0, s)
    rows = lib.vae2_conv2d_bwd_data_bnpart_rows(dyp, ctypes.byref(dyd), ctypes.byref(dxd), 3, 1, 1)
    assert rows > 0
    part = torch.empty(2 * rows * c, device=DEV)
    call("vae2_conv2d_bwd_data_bnpart", dyp, ctypes.byref(dyd), ops.ptr(wp1), ops.ptr(dx2),
         ctypes.byref(dxd), 3, 1, 1, xp, ctypes.byref(xd), ops.ptr(save), 1, ops.ptr(part), s)
    rows_r = lib.vae2_bn_partial_rows(ctypes.byref(xd))
    part_r = torch.empty(2 * rows_r * c, device=DEV)
    dx1p, dx1d = ops.act_of(dx1)
    call("vae2_bn_relu_bwd_reduce", dx1p, ctypes.byref(dx1d), None, ctypes.byref(xd), xp,
         ctypes.byref(xd), ops.ptr(save), 1, ops.ptr(part_r), s)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.equal(dw1, dw2)
    assert torch.equal(dx1, dx2)
    got = part.view(2, rows, c).double().sum(1)
    ref = part_r.view(2, rows_r, c).double().sum(1)
    # fp64 reference of the same sums
    g = dx1.double().reshape(-1, c)
    xx = x.double().reshape(-1, c)
    mask = (xx * save[2 * c:3 * c].double() + save[3 * c:].double()) > 0
    g = torch.where(mask, g, torch.zeros_like(g))
    exact = torch.stack([g.sum(0), (g * (xx - mean.double()) * invstd.double()).sum(0)])
    assert rel(got, exact) < 1e-5
    assert rel(ref, exact) < 1e-5


def _bottleneck_run(flags, monkeypatch, shape=(2, 64, 128), seed=3):
    """Bottleneck(64 -> 4 x 64, downsample) = layer1's first block, training BN."""
    from vae2 import hrnet, ops
    lazy, resbn = flags
    monkeypatch.setattr(ops, "LAZY_BN", lazy)
    monkeypatch.setattr(ops, "RES_BN", resbn)
    monkeypatch.setattr(ops, "MASK_BYTES", resbn)
    torch.manual_seed(seed)
    blk = hrnet.make_layer(hrnet.Bottleneck, 64, 64, 2).to(DEV)
    for m in blk.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.normal_(m.weight, 1.0, 0.3)
            nn.init.normal_(m.bias, 0.0, 0.3)
        elif isinstance(m, nn.Conv2d):
            nn.init.normal_(m.weight, 0.0, (2.0 / m.weight[0].numel()) ** 0.5)
    n, h, w = shape
    torch.manual_seed(seed + 1)
    x = ops.new_act((n, h, w, 64), torch.empty(1, device=DEV))
    with torch.no_grad():
        x.normal_()
    x.requires_grad_(True)
    y = hrnet.run_seq(blk, x)
    torch.manual_seed(seed + 2)
    torch.autograd.backward([y], [torch.randn_like(y)])
    torch.cuda.synchronize()
    return blk, x, y


@pytest.mark.parametrize("shape", [(2, 64, 128), (3, 40, 72)])
def test_resbn_shortcut_equals_stored(shape, monkeypatch):
    """ops.ResBN (the Bottleneck's downsample BN added inside bn3's apply, its partials and
    input gradient from bn3's backward kernels), the Bottleneck's LazyBN bn1 and bn3's ReLU
    mask bytes against the stored path: forward bit-identical, gradients and running
    statistics within fp32 summation-order noise."""
    from test_bench_instances_gpu import Recorder
    with Recorder() as rec:
        ba, xa, ya = _bottleneck_run((True, True), monkeypatch, shape)
    names = {k for _, _, ks in rec.calls for k in ks}
    # bn3's backward kernels specialised for the residual BatchNorm (RB = true) ran
    import re
    for rx in (r"bn_bwd_reduce_multi_kernel<\d+, true>", r"bn_bwd_apply_multi_kernel<\d+, true, "):
        assert any(re.match(rx, k) for k in names), (rx, sorted(names))
    bb, xb, yb = _bottleneck_run((False, False), monkeypatch, shape)
    assert torch.equal(ya, yb)
    assert rel_nz(xa.grad, xb.grad) < 1e-5
    for (na, pa), (_, pb) in zip(ba.named_parameters(), bb.named_parameters()):
        assert rel_nz(pa.grad, pb.grad) < 1e-5, na
    for (na, ra), (_, rb_) in zip(ba.named_buffers(), bb.named_buffers()):
        if "running" in na:
            assert torch.equal(ra, rb_), na


def _module_run(fuse_lazy, monkeypatch, seed=4):
    """A W18 stage-4 HighResolutionModule (4 branches, 2 BasicBlocks each, fuse rows with up
    paths and down chains) at 32x64, B=2, training BN."""
    from helpers import build, make_cfg
    from vae2 import ops
    monkeypatch.setattr(ops, "FUSE_LAZY", fuse_lazy)
    ed, _ = build(make_cfg(arch="w18", hw=(32, 64)))
    mod = ed.stage4[0].to(DEV)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in mod.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) / m.weight[0].numel() ** 0.5)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.copy_(1.0 + 0.3 * torch.randn(m.weight.shape, generator=g))
                m.bias.copy_(0.3 * torch.randn(m.bias.shape, generator=g))
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
    return mod, xs, ys


def test_fuse_lazy_units_equal_stored(monkeypatch):
    """The fuse units' BN outputs formed inside the fuse sum (ops.fuse_sum_relu lazies:
    vae2_fuse_sum_relu_bn) against the stored path: outputs bit-identical, input / weight
    / BN gradients within summation-order noise, running statistics identical."""
    ma, xa, ya = _module_run(True, monkeypatch)
    mb, xb, yb = _module_run(False, monkeypatch)
    for u, v in zip(ya, yb):
        assert torch.equal(u, v)
    for u, v in zip(xa, xb):
        assert rel_nz(u.grad, v.grad) < 1e-5
    for (n, p), (_, q) in zip(ma.named_parameters(), mb.named_parameters()):
        assert rel_nz(p.grad, q.grad) < 1e-5, n
    for (n, a), (_, b) in zip(ma.named_buffers(), mb.named_buffers()):
        if "running" in n:
            assert torch.equal(a, b), n
