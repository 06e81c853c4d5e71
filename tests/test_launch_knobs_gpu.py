"""Launch-shape knobs (vae2_conv2d_set_tune) change how work is partitioned, never what is
computed: a W18 stage-4 HighResolutionModule (enc_hrnet.py:177-262; four branches, fuse rows
with up- and down-sampling chains) forward + backward under each non-default setting against
the defaults.  Knobs that only re-schedule identical per-chunk work give bit-identical
results (key 20: the BatchNorm apply kernels striding over their pixel chunks); knobs that
re-partition a reduction (split counts, partial-statistics rows, row tiles, K splits) agree
to fp32 summation-order noise."""
import pytest
import torch
import torch.nn as nn

from helpers import build, make_cfg, rel_nz

pytestmark = pytest.mark.gpu
DEV = "cuda"

KNOBS = [
    # key, value, bit-identical
    (20, 1280, True),    # BN apply kernels: whole-round grid-stride (resident budget 1,280)
    (20, 64, True),      # ... and a budget that makes every workgroup walk many chunks
    (19, 2048, False),   # BN blocks per layer (partial-statistics rows)
    (19, 256, False),
    (18, 2048, False),   # gather weight-gradient splits
    (16, 1, False),      # narrow weight gradient: one tile per partial slab
    (17, 2, False),      # streaming 3x3: at least 2 steps per band
    (0, 0, False),       # gather GEMM: the 4-row-tile rule alone
    (15, 0, False),      # direct 3x3: no K split over 8 waves
    (15, 2, False),      # ... or over 16 waves (4 K shares)
    (21, 0, True),       # fuse sum + ReLU a channel per thread instead of a quad
]


def _run(seed=4):
    torch.manual_seed(seed)
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
    from vae2 import ops
    xs = []
    for c, h, w in [(18, 64, 128), (36, 32, 64), (72, 16, 32), (144, 8, 16)]:
        x = ops.new_act((4, h, w, c), torch.empty(1, device=DEV))
        with torch.no_grad():
            x.copy_(torch.randn(x.shape, generator=g).to(DEV))
        xs.append(x.requires_grad_(True))
    ys = mod.run(xs)
    gs = [torch.randn(y.shape, generator=g).to(DEV) for y in ys]
    torch.autograd.backward(ys, gs)
    torch.cuda.synchronize()
    return ([y.detach().clone() for y in ys], [x.grad.clone() for x in xs],
            {n: p.grad.clone() for n, p in mod.named_parameters()},
            {n: b.clone() for n, b in mod.named_buffers() if "running" in n})


@pytest.mark.parametrize("key,val,exact", KNOBS)
def test_knob_gives_the_default_result(key, val, exact):
    from vae2 import _lib
    lib = _lib.load()
    base = _run()
    prev = lib.vae2_conv2d_set_tune(key, val)
    assert prev >= 0, (key, val)
    try:
        alt = _run()
    finally:
        lib.vae2_conv2d_set_tune(key, prev)
    ys, dxs, dws, bufs = base
    ys2, dxs2, dws2, bufs2 = alt
    for a, b in zip(ys, ys2):
        assert torch.equal(a, b) if exact else rel_nz(b, a) < 1e-5
    for a, b in zip(dxs, dxs2):
        assert torch.equal(a, b) if exact else rel_nz(b, a) < 1e-5
    for n in dws:
        assert torch.equal(dws[n], dws2[n]) if exact else rel_nz(dws2[n], dws[n]) < 1e-5, n
    for n in bufs:
        assert torch.equal(bufs[n], bufs2[n]) if exact else rel_nz(bufs2[n], bufs[n]) < 1e-5, n


def test_knob_range_checks():
    """Out-of-range values are rejected (-1) and leave the setting unchanged."""
    from vae2 import _lib
    lib = _lib.load()
    for key, bad in [(15, 3), (16, 0), (16, 3), (17, 0), (17, 3), (18, 100), (19, 100000),
                     (20, -1)]:
        before = lib.vae2_conv2d_set_tune(key, {15: 1, 16: 2, 17: 1, 18: 1024, 19: 1024, 20: 0}[key])
        assert lib.vae2_conv2d_set_tune(key, bad) == -1, (key, bad)
        lib.vae2_conv2d_set_tune(key, before)
