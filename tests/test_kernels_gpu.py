"""Per-operator numerics of the HIP kernels (through vae2.ops) against plain
PyTorch fp32 CPU references of the same ops, forward and backward."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from helpers import rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 2e-5  # fp32 MFMA (exact fma chains) vs oneDNN: reduction-order differences only


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2)


CONV_SHAPES = [
    # N, H, W, Cin, Cout, k, stride, bias
    (2, 16, 16, 18, 18, 3, 1, False),
    (2, 17, 13, 9, 64, 3, 1, False),
    (2, 16, 16, 36, 72, 3, 2, False),
    (2, 15, 15, 18, 36, 3, 2, False),
    (2, 8, 8, 270, 270, 1, 1, True),
    (3, 1, 1, 270, 512, 1, 1, True),
    (2, 12, 20, 256, 18, 3, 1, False),
    (2, 16, 16, 64, 256, 1, 1, False),
    (2, 9, 9, 5, 7, 1, 2, False),
    (2, 8, 8, 154, 144, 3, 1, False),
    (2, 32, 64, 64, 64, 3, 1, False),
    (2, 8, 8, 270, 3, 1, 1, True),
    (1, 128, 512, 72, 270, 1, 1, True),   # M = 65536: the wide-N 1x1 tiles (2 x 9)
    (1, 64, 1024, 40, 130, 1, 1, False),  # wide, 9 tiles in one block
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd_bwd(shape):
    from vae2 import ops
    torch.manual_seed(0)
    n, h, w, cin, cout, k, s, bias = shape
    conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=bias)
    x = torch.randn(n, cin, h, w, requires_grad=True)
    y_ref = conv(x)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    # device copy; input given as a channel slice of a wider NHWC buffer
    cg = nn.Conv2d(cin, cout, k, s, k // 2, bias=bias).to(DEV)
    cg.load_state_dict(conv.state_dict())
    big = torch.zeros(n, h, w, cin + 5, device=DEV)
    big[..., 2:2 + cin] = nhwc(x.detach()).to(DEV)
    xg = big[..., 2:2 + cin].requires_grad_(True)
    yg = ops.conv(xg, cg)
    yg.backward(nhwc(gy).to(DEV))
    torch.cuda.synchronize()
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(nchw(xg.grad), x.grad) < TOL
    assert rel(cg.weight.grad, conv.weight.grad) < TOL
    if bias:
        assert rel(cg.bias.grad, conv.bias.grad) < TOL


DIRECT_SHAPES = [
    # N, H, W, Cin, Cout, bias: 3x3 / stride 1 / pad 1 through the LDS-tiled kernel
    (2, 16, 32, 18, 18, False),   # one slab (5 quads), padded channel quad
    (2, 13, 40, 36, 36, True),    # partial row and column tiles, 2 slabs
    (1, 8, 64, 64, 64, False),    # 2 slabs of 8 quads, TN = 4
    (2, 5, 7, 3, 5, False),       # image smaller than one tile, TM = 2
    (1, 8, 32, 154, 144, False),  # 5 slabs (39 quads), N split over 3 blocks
    (2, 6, 33, 256, 18, True),    # 8 slabs, 2 column tiles of which one has 1 column
    (2, 16, 32, 72, 72, False),   # weight gradient: 2 co slabs of 32 MFMA + 4 VALU rows
    # 1x1 (the direct weight-gradient kernel's KS = 1 form; data paths: gather kernel)
    (2, 8, 40, 270, 270, True, 1),
    (1, 4, 64, 64, 256, False, 1),
    (1, 5, 48, 18, 5, False, 1),
]


@pytest.mark.parametrize("shape", DIRECT_SHAPES)
def test_direct_conv3x3(shape):
    from vae2 import _lib, ops
    torch.manual_seed(3)
    n, h, w, cin, cout, bias = shape[:6]
    k = shape[6] if len(shape) > 6 else 3
    conv = nn.Conv2d(cin, cout, k, 1, k // 2, bias=bias)
    x = torch.randn(n, cin, h, w, requires_grad=True)
    y_ref = conv(x)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    cg = nn.Conv2d(cin, cout, k, 1, k // 2, bias=bias).to(DEV)
    cg.load_state_dict(conv.state_dict())
    lib = _lib.load()
    prev = lib.vae2_conv2d_set_algo(2)
    try:
        xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
        with torch.no_grad():
            xg.copy_(nhwc(x.detach()).to(DEV))
        xg.requires_grad_(True)
        dyg = ops.new_act((n, h, w, cout), xg)
        with torch.no_grad():
            dyg.copy_(nhwc(gy).to(DEV))
        yg = ops.conv(xg, cg)
        yg.backward(dyg)
        torch.cuda.synchronize()
        if k == 3:
            name = ctypes_name(xg, (n, h, w, cout))
            assert name.startswith(("dconv3_kernel", "dconv3s_kernel")), name
    finally:
        lib.vae2_conv2d_set_algo(prev)
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(nchw(xg.grad), x.grad) < TOL
    assert rel(cg.weight.grad, conv.weight.grad) < TOL
    if bias:
        assert rel(cg.bias.grad, conv.bias.grad) < TOL


REMAINDER_SHAPES = [
    # N, H, W, Cin, Cout, bias: 18 / 36 / 72-channel outputs (forward) and inputs (data
    # gradient) as 16*TN MFMA columns + NR VALU channels, 8-row (TM 4) and 4-row tiles
    (8, 128, 256, 18, 18, False),  # TM 4, NR 2 both directions
    (8, 64, 128, 36, 36, True),    # TM 2, NR 4 (two lanes per pixel)
    (2, 32, 64, 72, 72, False),    # TM 2, NR 8
    (4, 64, 96, 36, 18, False),    # forward NR 2, data gradient NR 4
    (2, 13, 40, 18, 36, True),     # partial row / column tiles
]


@pytest.mark.parametrize("shape", REMAINDER_SHAPES)
def test_direct_conv3x3_valu_remainder(shape):
    """dconv3 with the VALU remainder (vae2_conv2d_set_algo bit 16 clear): forward, data
    gradient, weight gradient and the BN-statistics epilogue against PyTorch, and the
    remainder instances are the ones launched."""
    from vae2 import _lib, ops
    torch.manual_seed(5)
    n, h, w, cin, cout, bias = shape
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=bias)
    x = torch.randn(n, cin, h, w, requires_grad=True)
    y_ref = conv(x)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    cg = nn.Conv2d(cin, cout, 3, 1, 1, bias=bias).to(DEV)
    cg.load_state_dict(conv.state_dict())
    from test_bench_instances_gpu import Recorder
    lib = _lib.load()
    prev = lib.vae2_conv2d_set_algo(2)
    try:
        xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
        with torch.no_grad():
            xg.copy_(nhwc(x.detach()).to(DEV))
        xg.requires_grad_(True)
        gpad = ops.new_act((n, h, w, cout), xg)  # padded pixel stride, as in the model
        with torch.no_grad():
            gpad.copy_(nhwc(gy).to(DEV))
        with Recorder() as rec:  # launch log read in the calling thread (autograd's too)
            yg = ops.conv(xg, cg)
            yg.backward(gpad)
            torch.cuda.synchronize()
        names = [k for _, _, ks in rec.calls for k in ks]
        # BN statistics from the remainder epilogue (conv_bn: running mean / var)
        bn, bg = nn.BatchNorm2d(cout, momentum=0.5), nn.BatchNorm2d(cout, momentum=0.5).to(DEV)
        with torch.no_grad():
            ops.conv_bn(xg.detach(), cg, bg, relu=False)
            bn(conv(x.detach()))
        torch.cuda.synchronize()
    finally:
        lib.vae2_conv2d_set_algo(prev)
    for c in (cout, cin):
        nr = c % 16
        if nr in (2, 4, 8) and c // 16 in (1, 2, 4):
            # dconv3_kernel<TM, TN, FLIP, BF, NR, BNX> or (18 -> 18, 36 -> 36: the
            # streaming kernel) dconv3s_kernel<TN, NR, Q, FLIP, BNX>
            assert any((k.startswith("dconv3_kernel") and k[:-1].split(", ")[4:5] == [str(nr)]) or
                       (k.startswith("dconv3s_kernel") and k[:-1].split(", ")[1:2] == [str(nr)])
                       for k in names), (c, names)
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(nchw(xg.grad), x.grad) < TOL
    assert rel(cg.weight.grad, conv.weight.grad) < TOL
    if bias:
        assert rel(cg.bias.grad, conv.bias.grad) < TOL
    assert rel(bg.running_mean, bn.running_mean) < 1e-5
    assert rel(bg.running_var, bn.running_var) < 1e-5


@pytest.mark.parametrize("cout", [18, 36])
def test_valu_remainder_equals_padded_tiles(cout):
    """The remainder path (bit 16 clear) and the all-MFMA padded tiles (bit 16 set) compute
    the same conv: equal up to fp32 summation order."""
    from vae2 import _lib, ops
    torch.manual_seed(8)
    lib = _lib.load()
    x = ops.new_act((8, 64, 128, 36), torch.empty(1, device=DEV))
    x.normal_()
    w = torch.randn(cout, 36, 3, 3, device=DEV) * 0.05
    outs = []
    prev = lib.vae2_conv2d_set_algo(2)
    try:
        for algo in (2, 2 + 16):
            lib.vae2_conv2d_set_algo(algo)
            conv = nn.Conv2d(36, cout, 3, 1, 1, bias=False).to(DEV)
            with torch.no_grad():
                conv.weight.copy_(w)
                outs.append(ops.conv(x, conv).clone())
    finally:
        lib.vae2_conv2d_set_algo(prev)
    assert rel(outs[0], outs[1]) < 1e-6


BF16_SHAPES = [
    # N, H, W, Cin, Cout, k, stride, bias, algo: every conv kernel with bf16 operands
    (2, 16, 32, 18, 18, 3, 1, False, 2),    # direct 3x3 (dconv3 fwd / dgrad, wgrad3)
    (2, 13, 40, 36, 36, 3, 1, True, 2),     # partial tiles, 2 slabs
    (1, 8, 32, 154, 144, 3, 1, False, 2),   # 5 slabs, N split
    (2, 17, 13, 9, 64, 3, 1, False, 1),     # gather kernel (igemm), channel-pad quad
    (2, 16, 16, 36, 72, 3, 2, False, 0),    # stride 2 (igemm, parity-class dgrad, wgrad)
    (2, 8, 8, 270, 270, 1, 1, True, 0),     # 1x1
    (1, 128, 512, 72, 270, 1, 1, True, 0),  # wide-N 1x1 tiles
    (2, 12, 20, 256, 18, 3, 1, False, 0),   # K split
]


@pytest.mark.parametrize("shape", BF16_SHAPES)
def test_conv_bf16_operands(shape):
    """vae2_conv2d_set_mfma_bf16(1): every conv kernel rounds its MFMA operands to bf16
    (RNE) and accumulates in fp32, so forward, data gradient and weight gradient equal
    the fp64 conv of the bf16-rounded x, w and dy up to fp32 summation order."""
    from vae2 import _lib, ops
    torch.manual_seed(4)
    n, h, w, cin, cout, k, s, bias, algo = shape
    conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=bias)
    x = torch.randn(n, cin, h, w)
    ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
    gy = torch.randn(n, cout, ho, wo)

    def bf(t):
        return t.bfloat16().double()
    x64 = bf(x).requires_grad_(True)
    w64 = bf(conv.weight.detach()).requires_grad_(True)
    b64 = conv.bias.detach().double() if bias else None
    y64 = F.conv2d(x64, w64, b64, s, k // 2)
    y64.backward(bf(gy))
    cg = nn.Conv2d(cin, cout, k, s, k // 2, bias=bias).to(DEV)
    cg.load_state_dict(conv.state_dict())
    lib = _lib.load()
    prev_algo = lib.vae2_conv2d_set_algo(algo)
    prev_bf = lib.vae2_conv2d_set_mfma_bf16(1)
    try:
        xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
        with torch.no_grad():
            xg.copy_(nhwc(x).to(DEV))
        xg.requires_grad_(True)
        yg = ops.conv(xg, cg)
        yg.backward(nhwc(gy).to(DEV))
        torch.cuda.synchronize()
    finally:
        lib.vae2_conv2d_set_mfma_bf16(prev_bf)
        lib.vae2_conv2d_set_algo(prev_algo)
    tol = 3e-5
    assert rel(nchw(yg).double(), y64) < tol
    assert rel(nchw(xg.grad).double(), x64.grad) < tol
    assert rel(cg.weight.grad.double(), w64.grad) < tol
    if bias:
        assert rel(cg.bias.grad.double(), gy.double().sum((0, 2, 3))) < tol
    # and the bf16 rounding itself is visible against the fp32 conv (the path ran)
    y32 = F.conv2d(x, conv.weight.detach(), conv.bias.detach() if bias else None, s, k // 2)
    assert rel(nchw(yg).cpu(), y32) > 1e-4


def ctypes_name(x, yshape):
    from vae2 import ops, prof
    _, xa = ops.act_of(x)
    return prof.fwd_kernel_name(xa, yshape, 3, 1, 1)


def test_multi_bn_equals_per_layer():
    """conv_bn_multi (independent layers of one depth level sharing every BatchNorm
    launch) == the same layers one by one, bit for bit: outputs, input / residual /
    parameter gradients and running statistics."""
    from vae2 import ops
    torch.manual_seed(6)
    shapes = [(2, 16, 32, 18, 18), (2, 8, 16, 36, 36), (2, 4, 8, 72, 72), (2, 2, 4, 144, 144),
              (2, 16, 32, 18, 36), (2, 8, 16, 36, 72), (2, 4, 8, 72, 144)]  # 7 > 6: two launches

    def make(seed):
        torch.manual_seed(seed)
        layers = []
        for n, h, w, ci, co in shapes:
            conv = nn.Conv2d(ci, co, 3, 1, 1, bias=False).to(DEV)
            bn = nn.BatchNorm2d(co, momentum=0.01).to(DEV)
            nn.init.normal_(bn.weight, 1.0, 0.2)
            nn.init.normal_(bn.bias, 0.0, 0.2)
            layers.append((conv, bn))
        xs = [ops.new_act((n, h, w, ci), torch.empty(1, device=DEV)) for n, h, w, ci, co in shapes]
        rs = [ops.new_act((n, h, w, co), xs[0]) for n, h, w, ci, co in shapes]
        for t in xs + rs:
            with torch.no_grad():
                t.normal_()
            t.requires_grad_(True)
        return layers, xs, rs

    la, xa, ra = make(7)
    lb, xb, rb = make(7)
    ya = ops.conv_bn_multi(xa, [c for c, _ in la], [b for _, b in la], True,
                           residuals=[r if i % 2 else None for i, r in enumerate(ra)])
    yb = [ops.conv_bn(x, c, b, True, r if i % 2 else None)
          for i, ((c, b), x, r) in enumerate(zip(lb, xb, rb))]
    gs = [torch.randn_like(y) for y in ya]
    torch.autograd.backward(ya, gs)
    torch.autograd.backward(yb, gs)
    torch.cuda.synchronize()
    for u, v in zip(ya, yb):
        assert torch.equal(u, v)
    for u, v in zip(xa + [r for i, r in enumerate(ra) if i % 2],
                    xb + [r for i, r in enumerate(rb) if i % 2]):
        assert torch.equal(u.grad, v.grad)
    for (ca, ba), (cb, bb) in zip(la, lb):
        for p, q in ((ca.weight, cb.weight), (ba.weight, bb.weight), (ba.bias, bb.bias)):
            assert torch.equal(p.grad, q.grad)
        assert torch.equal(ba.running_mean, bb.running_mean)
        assert torch.equal(ba.running_var, bb.running_var)


@pytest.mark.parametrize("cin,cout,h,w", [(18, 18, 16, 32), (64, 36, 12, 40)])
def test_direct_conv3x3_bn_stats(cin, cout, h, w):
    """BN statistics from the direct kernel's epilogue (its own partial-row count)."""
    from vae2 import _lib, ops
    torch.manual_seed(4)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
    bn = nn.BatchNorm2d(cout, momentum=0.01)
    x = torch.randn(2, cin, h, w)
    y_ref = F.relu(bn(conv(x)))
    cg, bg = nn.Conv2d(cin, cout, 3, 1, 1, bias=False).to(DEV), nn.BatchNorm2d(cout, momentum=0.01).to(DEV)
    cg.load_state_dict(conv.state_dict())
    lib = _lib.load()
    prev = lib.vae2_conv2d_set_algo(2)
    try:
        xg = ops.new_act((2, h, w, cin), torch.empty(1, device=DEV))
        xg.copy_(nhwc(x).to(DEV))
        yg = ops.conv_bn(xg, cg, bg, relu=True)
        torch.cuda.synchronize()
    finally:
        lib.vae2_conv2d_set_algo(prev)
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(bg.running_mean, bn.running_mean) < 1e-5
    assert rel(bg.running_var, bn.running_var) < 1e-5


@pytest.mark.parametrize("relu,res,stride,cout", [
    (True, False, 1, 36), (False, False, 2, 36), (True, True, 1, 36),
    # channel-quad kernels: padded last quad (18 -> 20, 7 -> 8, 5 -> 8), wide (270: 68 quads)
    (True, False, 1, 18), (True, True, 1, 18), (True, False, 1, 270), (True, True, 2, 5),
    (True, True, 1, 7),
    # residual as an unaligned channel slice: the scalar fallback
    (True, "view", 1, 18)])
def test_conv_bn_train(relu, res, stride, cout):
    from vae2 import ops
    torch.manual_seed(1)
    n, h, w, cin = 4, 12, 10, 18
    conv = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
    bn = nn.BatchNorm2d(cout, momentum=0.01)
    nn.init.normal_(bn.weight, 1.0, 0.2)
    nn.init.normal_(bn.bias, 0.0, 0.2)
    conv_g, bn_g = conv.to(DEV), bn.to(DEV)
    conv_c = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
    conv_c.load_state_dict({k: v.cpu() for k, v in conv_g.state_dict().items()})
    bn_c = nn.BatchNorm2d(cout, momentum=0.01)
    bn_c.load_state_dict({k: v.cpu() for k, v in bn_g.state_dict().items()})
    x = torch.randn(n, cin, h, w, requires_grad=True)
    oh = (h - 1) // stride + 1
    ow = (w - 1) // stride + 1
    r = torch.randn(n, cout, oh, ow, requires_grad=True) if res else None
    y_ref = bn_c(conv_c(x))
    if res:
        y_ref = y_ref + r
    if relu:
        y_ref = F.relu(y_ref)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    xg = nhwc(x.detach()).to(DEV).requires_grad_(True)
    if res == "view":
        wide = torch.zeros(n, oh, ow, cout + 3, device=DEV)
        wide[..., 1:1 + cout] = nhwc(r.detach()).to(DEV)
        rg = wide[..., 1:1 + cout].requires_grad_(True)
    else:
        rg = nhwc(r.detach()).to(DEV).requires_grad_(True) if res else None
    yg = ops.conv_bn(xg, conv_g, bn_g, relu=relu, residual=rg)
    yg.backward(nhwc(gy).to(DEV))
    torch.cuda.synchronize()
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(nchw(xg.grad), x.grad) < 1e-4
    assert rel(conv_g.weight.grad, conv_c.weight.grad) < 1e-4
    assert rel(bn_g.weight.grad, bn_c.weight.grad) < 1e-4
    assert rel(bn_g.bias.grad, bn_c.bias.grad) < 1e-5
    if res:
        assert rel(nchw(rg.grad), r.grad) < 1e-5
    assert rel(bn_g.running_mean, bn_c.running_mean) < 1e-5
    assert rel(bn_g.running_var, bn_c.running_var) < 1e-5
    assert int(bn_g.num_batches_tracked) == int(bn_c.num_batches_tracked) == 1


@pytest.mark.parametrize("aligned", [True, False])
def test_conv_bn_residual_link_accumulates(aligned):
    """A residual whose GradLink buffer already holds the other consumer's gradient: the
    BN backward apply sums its residual gradient onto that buffer in-kernel
    (vae2_bn_layer.dres_acc: the multi-layer path, aligned residual) or with an add (the
    per-layer path an unaligned residual view takes); either way the residual's gradient
    is the reference's plus the prefilled contribution."""
    from vae2 import ops
    torch.manual_seed(2)
    n, h, w, c = 2, 10, 12, 18
    conv = nn.Conv2d(c, c, 3, 1, 1, bias=False)
    bn = nn.BatchNorm2d(c, momentum=0.01)
    nn.init.normal_(bn.weight, 1.0, 0.2)
    x = torch.randn(n, c, h, w, requires_grad=True)
    r = torch.randn(n, c, h, w, requires_grad=True)
    y_ref = F.relu(bn(conv(x)) + r)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    other = torch.randn(n, h, w, c)
    conv_g, bn_g = nn.Conv2d(c, c, 3, 1, 1, bias=False).to(DEV), nn.BatchNorm2d(c, momentum=0.01).to(DEV)
    conv_g.load_state_dict(conv.state_dict())
    bn_g.load_state_dict(bn.state_dict())
    xg = ops.new_act((n, h, w, c), torch.empty(1, device=DEV))
    rg = (ops.new_act((n, h, w, c), xg) if aligned
          else torch.zeros(n, h, w, c + 3, device=DEV)[..., 1:1 + c])
    assert ops._bn_quad_ok(rg) == aligned
    with torch.no_grad():
        xg.copy_(nhwc(x.detach()).to(DEV))
        rg.copy_(nhwc(r.detach()).to(DEV))
    rg.requires_grad_(True)
    link = ops.GradLink(2)
    link.buf = ops.new_act((n, h, w, c), xg)
    with torch.no_grad():
        link.buf.copy_(other.to(DEV))
    link.done = 1  # the other consumer's backward ran first and handed the buffer on
    yg = ops.conv_bn_multi([xg], [conv_g], [bn_g], True, residuals=[rg], res_links=[link])[0]
    yg.backward(nhwc(gy).to(DEV))
    torch.cuda.synchronize()
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(rg.grad.cpu(), nhwc(r.grad) + other) < 1e-5
    assert rel(conv_g.weight.grad, conv.weight.grad) < 1e-4


KS_SHAPES = [
    # N, H, W, Cin, Cout, k, stride: the gather kernel's in-workgroup K split (KS = 4:
    # >= 16 K chunks and < 512 workgroups), its BN-statistics epilogue, and stride-2
    # data gradients (parity classes, some with no valid tap) accumulated with beta = 1
    (2, 8, 8, 144, 144, 3, 1),
    (1, 16, 16, 144, 72, 3, 2),
    (2, 6, 10, 72, 144, 3, 2),
    (4, 4, 4, 270, 144, 1, 1),
]


@pytest.mark.parametrize("shape", KS_SHAPES)
@pytest.mark.parametrize("ksplit", [True, False])
def test_igemm_ksplit_conv_bn_and_accumulating_dgrad(shape, ksplit):
    """conv_bn (training) through the gather kernel with the K split on and off
    (vae2_conv2d_set_algo bit 8): output, BN running statistics (the KS epilogue's
    per-tile rows), input / weight / BN gradients against PyTorch; then the data
    gradient accumulated onto a prefilled buffer (beta = 1, the GradLink path)."""
    import ctypes
    from vae2 import _lib, ops
    torch.manual_seed(2)
    n, h, w, cin, cout, k, s = shape
    pad = k // 2
    conv = nn.Conv2d(cin, cout, k, s, pad, bias=False)
    bn = nn.BatchNorm2d(cout, momentum=0.01)
    nn.init.normal_(bn.weight, 1.0, 0.2)
    nn.init.normal_(bn.bias, 0.0, 0.2)
    conv_g = nn.Conv2d(cin, cout, k, s, pad, bias=False).to(DEV)
    conv_g.load_state_dict(conv.state_dict())
    bn_g = nn.BatchNorm2d(cout, momentum=0.01).to(DEV)
    bn_g.load_state_dict(bn.state_dict())
    x = torch.randn(n, cin, h, w, requires_grad=True)
    y_ref = F.relu(bn(conv(x)))
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    lib = _lib.load()
    prev = lib.vae2_conv2d_set_algo(1 | (0 if ksplit else 8))
    try:
        xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
        with torch.no_grad():
            xg.copy_(nhwc(x.detach()).to(DEV))
        xg.requires_grad_(True)
        yg = ops.conv_bn(xg, conv_g, bn_g, relu=True)
        yg.backward(nhwc(gy).to(DEV))
        torch.cuda.synchronize()
        assert rel(nchw(yg), y_ref) < TOL
        assert rel(nchw(xg.grad), x.grad) < 1e-4
        assert rel(conv_g.weight.grad, conv.weight.grad) < 1e-4
        assert rel(bn_g.weight.grad, bn.weight.grad) < 1e-4
        assert rel(bn_g.bias.grad, bn.bias.grad) < 1e-5
        assert rel(bn_g.running_mean, bn.running_mean) < 1e-5
        assert rel(bn_g.running_var, bn.running_var) < 1e-5
        # data gradient onto a prefilled buffer (beta = 1)
        oh, ow = y_ref.shape[2:]
        dyc = torch.randn(n, cout, oh, ow)
        pre = torch.randn(n, cin, h, w)
        xr = torch.zeros(n, cin, h, w, requires_grad=True)
        F.conv2d(xr, conv.weight.detach(), None, s, pad).backward(dyc)
        dy = ops.new_act((n, oh, ow, cout), xg)
        dx = ops.new_act((n, h, w, cin), xg)
        with torch.no_grad():
            dy.copy_(nhwc(dyc).to(DEV))
            dx.copy_(nhwc(pre).to(DEV))
        dyp, dya = ops.act_of(dy)
        dxp, dxa = ops.act_of(dx)
        wp = ops.packed_weight(conv_g.weight, 1)
        ops.call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dya), ops.ptr(wp), dxp,
                 ctypes.byref(dxa), k, s, pad, 1.0, ops.stream_ptr())
        torch.cuda.synchronize()
        assert rel(nchw(dx), xr.grad + pre) < TOL
    finally:
        lib.vae2_conv2d_set_algo(prev)


@pytest.mark.parametrize("shape", [
    # N, H, W, Cin, Cout, k, stride: forward N = Cout, data gradient N = Cin
    (2, 32, 64, 36, 18, 3, 1), (2, 32, 64, 18, 36, 3, 2), (2, 24, 40, 36, 36, 1, 1),
    (3, 17, 23, 18, 18, 3, 2)])
def test_igemm_valu_remainder(shape):
    """The gather kernel with 18 / 36 output channels as 16 + 2 / 32 + 4 (VALU remainder
    columns, vae2_conv2d_set_tune key 6; gather kernel only, K split off so it applies):
    conv_bn training output, running statistics (the remainder columns' partial rows),
    input / weight / BN gradients against PyTorch, and the data gradient accumulated onto
    a prefilled buffer (beta = 1), incl. the stride-2 parity classes."""
    from vae2 import _lib
    lib = _lib.load()
    prev_nr = lib.vae2_conv2d_set_tune(6, 1)
    try:
        test_igemm_ksplit_conv_bn_and_accumulating_dgrad(shape, False)
    finally:
        lib.vae2_conv2d_set_tune(6, prev_nr)


def test_conv_bn_eval():
    from vae2 import ops
    torch.manual_seed(2)
    conv = nn.Conv2d(8, 16, 3, 1, 1, bias=False)
    bn = nn.BatchNorm2d(16, momentum=0.01)
    bn.running_mean.normal_()
    bn.running_var.uniform_(0.5, 2.0)
    conv.eval(), bn.eval()
    x = torch.randn(2, 8, 9, 9)
    y_ref = F.relu(bn(conv(x)))
    cg, bg = nn.Conv2d(8, 16, 3, 1, 1, bias=False).to(DEV), nn.BatchNorm2d(16).to(DEV)
    cg.load_state_dict(conv.state_dict()), bg.load_state_dict(bn.state_dict())
    bg.eval()
    with torch.no_grad():
        yg = ops.conv_bn(nhwc(x).to(DEV), cg, bg, relu=True)
    assert rel(nchw(yg), y_ref) < TOL


@pytest.mark.parametrize("shapes", [[(16, 32), (8, 16), (4, 8), (2, 4)], [(9, 9), (5, 5), (3, 3)]])
def test_up_cat(shapes):
    from vae2 import ops
    torch.manual_seed(3)
    chans = [4, 8, 16, 32][:len(shapes)]
    xs = [torch.randn(2, c, h, w, requires_grad=True) for c, (h, w) in zip(chans, shapes)]
    hw = shapes[0]
    y_ref = torch.cat([xs[0]] + [F.interpolate(x, size=list(hw), mode="bilinear",
                                               align_corners=False) for x in xs[1:]], 1)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    xg = [nhwc(x.detach()).to(DEV).requires_grad_(True) for x in xs]
    yg = ops.up_cat(xg)
    yg.backward(nhwc(gy).to(DEV))
    assert rel(nchw(yg), y_ref) < 1e-6
    for a, b in zip(xg, xs):
        assert rel(nchw(a.grad), b.grad) < 1e-5


@pytest.mark.parametrize("c,sizes", [(8, [(16, 12), (16, 12), (8, 6), (2, 2)]),
                                     (18, [(16, 32), (8, 16), (2, 4), (1, 1)]),
                                     (18, [(32, 64), (16, 32), (8, 16), (4, 8)]),
                                     (36, [(16, 16), (8, 8), (4, 4)]),
                                     (6, [(8, 16), (4, 8)])])
@pytest.mark.parametrize("pow2", [True, False])
def test_fuse_sum_relu(c, sizes, pow2, monkeypatch):
    """Includes 18 channels (a padded channel quad in the vectorised adjoint), x8
    upsampling and a 1x1 source (a window wider than the adjoint's unrolled one); the
    exact 2/4/8 rows take vae2_upsample_bilinear_bwd_pow2 unless pow2 is off."""
    from vae2 import ops
    monkeypatch.setattr(ops, "UP_POW2", pow2)
    torch.manual_seed(4)
    hw = sizes[0]
    terms = [torch.randn(2, c, h, w, requires_grad=True) for h, w in sizes]
    y = terms[0]
    for tt in terms[1:]:
        y = y + (tt if tt.shape[-2:] == hw else F.interpolate(tt, size=list(hw), mode="bilinear"))
    y_ref = F.relu(y)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    tg = [nhwc(x.detach()).to(DEV).requires_grad_(True) for x in terms]
    yg = ops.fuse_sum_relu(tg, hw)
    yg.backward(nhwc(gy).to(DEV))
    assert rel(nchw(yg), y_ref) < 1e-6
    for a, b in zip(tg, terms):
        assert rel(nchw(a.grad), b.grad) < 1e-5


def test_upsample_bwd_pow2_betas_and_order():
    """The ABI directly: targets in any ratio order, beta accumulation, 1-pixel targets
    (both edge folds on one source), and -1 for a non power-of-two target."""
    import ctypes
    from vae2 import ops
    from vae2._lib import Act, call, load
    lib = load()
    torch.manual_seed(6)
    n, c, H, W = 2, 10, 8, 16
    dy = torch.randn(n, c, H, W)
    tshapes = [(2, 4), (8 // 2, 16 // 2), (1, 2)]  # ratios 4, 2, 8
    ref, prev, betas = [], [], [0.0, 1.0, 0.5]
    for (h, w), b in zip(tshapes, betas):
        z = torch.zeros(n, c, h, w, requires_grad=True)
        F.interpolate(z, size=[H, W], mode="bilinear").backward(dy)
        p0 = torch.randn(n, c, h, w)
        prev.append(p0)
        ref.append(z.grad + b * p0)
    g = ops.new_act((n, H, W, c), torch.empty(0, device=DEV))
    g.copy_(nhwc(dy))
    dxs = []
    for p in prev:
        d = ops.new_act(tuple(nhwc(p).shape), g)
        d.copy_(nhwc(p))
        dxs.append(d)
    gp, ga = ops.act_of(g)
    views = [ops.act_of(d) for d in dxs]
    acts = (Act * 3)(*[a for _, a in views])
    wsz = lib.vae2_upsample_bilinear_bwd_pow2_ws_size(ctypes.byref(ga), 3, acts)
    assert wsz > 0
    ws = torch.empty(wsz, device=DEV)
    bt = (ctypes.c_float * 3)(*betas)
    ptrs = (ctypes.c_void_p * 3)(*[p for p, _ in views])
    call("vae2_upsample_bilinear_bwd_pow2", gp, ctypes.byref(ga), 3, ptrs, acts, bt,
         ws.data_ptr(), wsz, None)
    torch.cuda.synchronize()
    for d, r in zip(dxs, ref):
        assert rel(nchw(d), r) < 1e-6
    bad = (Act * 1)(Act(n, 3, 5, c, c))
    assert lib.vae2_upsample_bilinear_bwd_pow2_ws_size(ctypes.byref(ga), 1, bad) == -1


@pytest.mark.parametrize("c,H,W", [(18, 16, 64), (36, 40, 128), (72, 8, 64)])
def test_upsample_bwd_pow2_one_pass_route(c, H, W):
    """The fuse layers' pow2 adjoint routed through the heads' one-pass band kernel
    (targets 2 / 4 / 8 in order, 64-pixel rows; betas accumulate) against torch's adjoint,
    and against the two-pass form (vae2_heads_set_algo bit 2)."""
    import ctypes
    from vae2 import ops
    from vae2._lib import Act, call, load
    lib = load()
    torch.manual_seed(c + H)
    n = 2
    dy = torch.randn(n, c, H, W)
    betas = [0.0, 1.0, 0.5]
    ref, prev = [], []
    for s, b in enumerate(betas):
        z = torch.zeros(n, c, H >> (s + 1), W >> (s + 1), requires_grad=True)
        F.interpolate(z, size=[H, W], mode="bilinear").backward(dy)
        p0 = torch.randn(z.shape)
        prev.append(p0)
        ref.append(z.grad + b * p0)
    g = ops.new_act((n, H, W, c), torch.empty(0, device=DEV))
    g.copy_(nhwc(dy))
    gp, ga = ops.act_of(g)
    outs = []
    try:
        for algo in (64, 4):  # bit 6: the one-pass route (off by default); bit 2: two-pass
            lib.vae2_heads_set_algo(algo)
            dxs = []
            for p0 in prev:
                d = ops.new_act(tuple(nhwc(p0).shape), g)
                d.copy_(nhwc(p0))
                dxs.append(d)
            views = [ops.act_of(d) for d in dxs]
            acts = (Act * 3)(*[a for _, a in views])
            wsz = lib.vae2_upsample_bilinear_bwd_pow2_ws_size(ctypes.byref(ga), 3, acts)
            ws = torch.empty(wsz, device=DEV)
            bt = (ctypes.c_float * 3)(*betas)
            ptrs = (ctypes.c_void_p * 3)(*[p for p, _ in views])
            call("vae2_upsample_bilinear_bwd_pow2", gp, ctypes.byref(ga), 3, ptrs, acts, bt,
                 ws.data_ptr(), wsz, None)
            torch.cuda.synchronize()
            for d, r in zip(dxs, ref):
                assert rel(nchw(d), r) < 1e-6, (algo, rel(nchw(d), r))
            outs.append([d.cpu() for d in dxs])
    finally:
        lib.vae2_heads_set_algo(0)
    for a, b in zip(*outs):
        assert rel(a, b) < 1e-6


def test_cat_codemap_and_avgpool():
    from vae2 import ops
    torch.manual_seed(5)
    code = torch.randn(3, 4, 1, 1)
    z = torch.randn(3, 4, 1, 1, requires_grad=True)
    x = torch.randn(3, 6, 5, 7, requires_grad=True)
    y_ref = torch.cat([code.repeat(1, 1, 5, 7), z.repeat(1, 1, 5, 7), x], 1)
    p_ref = F.adaptive_avg_pool2d(y_ref, 1)
    gp = torch.randn_like(p_ref)
    p_ref.backward(gp)
    zg = nhwc(z.detach()).to(DEV).requires_grad_(True)
    xg = nhwc(x.detach()).to(DEV).requires_grad_(True)
    yg = ops.cat([nhwc(code).to(DEV), zg, xg], (5, 7), tiles=[True, True, False])
    pg = ops.avgpool(yg)
    pg.backward(nhwc(gp).to(DEV))
    assert rel(nchw(yg), y_ref.detach()) == 0.0
    assert rel(nchw(pg), p_ref) < 1e-6
    assert rel(nchw(zg.grad), z.grad) < 1e-5
    assert rel(nchw(xg.grad), x.grad) < 1e-6


def test_l1_reparam_kl_weighted_sum():
    from vae2 import ops
    torch.manual_seed(6)
    B, zc = 4, 10
    p = torch.randn(B, 9, 6, 8, requires_grad=True)
    tg = torch.randn(B, 9, 6, 8)
    mv = torch.randn(B, 2 * zc, 1, 1, requires_grad=True)
    eps = torch.randn(B, zc, 1, 1)
    mu, lv = mv[:, :zc], mv[:, zc:]
    z_ref = mu + torch.exp(torch.mul(lv, 0.5)) * eps
    l1_ref = torch.sum(torch.abs(p - tg)) / B
    kl_ref = torch.sum(0.5 * (mu ** 2 + torch.exp(lv) - lv - 1)) / B
    gz = torch.randn_like(z_ref)
    tot_ref = 1.0 * l1_ref + 0.5 * kl_ref + (z_ref * gz).sum()
    tot_ref.backward()

    pg = nhwc(p.detach()).to(DEV).requires_grad_(True)
    mvg = nhwc(mv.detach()).to(DEV).requires_grad_(True)
    zg, klg = ops.reparam_kl(mvg, nhwc(eps).to(DEV), scale=1.0 / B)
    l1g = ops.l1(pg, nhwc(tg).to(DEV), 1.0 / B)
    tot = ops.weighted_sum([l1g, klg], [1.0, 0.5])
    (tot + (nchw(zg) * gz.to(DEV)).sum()).backward()
    assert abs(float(l1g) - float(l1_ref)) <= 1e-6 * abs(float(l1_ref))
    assert abs(float(klg) - float(kl_ref)) <= 1e-6 * abs(float(kl_ref))
    assert rel(nchw(zg), z_ref) < 1e-6
    assert rel(nchw(pg.grad), p.grad) < 1e-6
    assert rel(nchw(mvg.grad), mv.grad) < 1e-6


def test_fused_adam_matches_torch():
    from vae2.optim import FusedAdam
    torch.manual_seed(7)
    m_ref = nn.Sequential(nn.Linear(33, 17), nn.Linear(17, 5))
    m_gpu = nn.Sequential(nn.Linear(33, 17), nn.Linear(17, 5)).to(DEV)
    m_gpu.load_state_dict(m_ref.state_dict())
    opt_ref = torch.optim.Adam(m_ref.parameters(), lr=1e-3)
    opt = FusedAdam([m_gpu], lr=1e-3)
    for step in range(3):
        grads = [torch.randn_like(p) for p in m_ref.parameters()]
        for p, g in zip(m_ref.parameters(), grads):
            p.grad = g.clone()
        for p, g in zip(m_gpu.parameters(), grads):
            p.main_grad.copy_(g)
        opt_ref.step()
        opt.step()
    for a, b in zip(m_gpu.parameters(), m_ref.parameters()):
        assert rel(a, b) < 1e-6
    sd = opt.state_dict()
    ref_sd = opt_ref.state_dict()
    for k in ref_sd["state"]:
        assert rel(sd["state"][k]["exp_avg"], ref_sd["state"][k]["exp_avg"]) < 1e-6


MULTI_SHAPES = [
    # N, H, W, Cin, Cout, k, bias: one depth level's independent convs
    (2, 16, 32, 18, 18, 3, False),
    (2, 13, 40, 36, 36, 3, True),
    (1, 8, 32, 154, 144, 3, False),
    (2, 5, 7, 3, 5, 3, False),
    (2, 16, 32, 18, 18, 3, True),
    (2, 8, 8, 36, 18, 1, False),   # 1x1: not a direct-3x3 job, issued on its own
    (2, 13, 40, 36, 36, 3, False),
]


def test_conv2d_multi_grouped_equals_single_calls():
    """vae2_conv2d_multi (direct-3x3 jobs sharing launches, grouped by tile shape) gives
    the single-call results bit for bit: forward outputs and BN partial statistics, and
    data gradients, including two data-gradient jobs accumulating into one output
    (beta 0 then 1: the second runs after the first's launch)."""
    import ctypes
    from vae2 import _lib, ops
    from vae2._lib import Act
    lib = _lib.load()
    prev = lib.vae2_conv2d_set_algo(2 + 16)  # (VALU-remainder layers are never grouped)
    prev_g = lib.vae2_conv2d_set_grouping(1)
    prev_k = lib.vae2_conv2d_set_tune(15, 0)  # (nor the K-split 8-wave form: own launches)
    s = ops.stream_ptr()
    torch.manual_seed(5)
    like = torch.empty(1, device=DEV)

    class Spec:
        def __init__(self, k):
            self.k, self.stride, self.pad = k, 1, k // 2
    try:
        L = []
        for (n, h, w, cin, cout, k, bias) in MULTI_SHAPES:
            x = ops.new_act((n, h, w, cin), like).normal_()
            dy = ops.new_act((n, h, w, cout), like).normal_()
            wt = torch.randn(cout, cin, k, k, device=DEV) * 0.1
            b = torch.randn(cout, device=DEV) if bias else None
            xp, xa = ops.act_of(x)
            rows = lib.vae2_conv2d_fwd_stats_rows(xp, ctypes.byref(xa),
                                                  ctypes.byref(Act(n, h, w, cout, cout)), k, 1,
                                                  k // 2)
            L.append(dict(x=x, dy=dy, w=wt, b=b, k=k, rows=rows, shape=(n, h, w, cin, cout),
                          w0=ops.packed_weight(wt, 0), w1=ops.packed_weight(wt, 1)))

        def run(grouped):
            outs, stats, dxs = [], [], []
            cg = ops.ConvGroup() if grouped else None
            for d in L:
                n, h, w, cin, cout = d["shape"]
                y = ops.new_act((n, h, w, cout), like)
                st = torch.empty(2 * d["rows"] * cout, device=DEV)
                xp, xa = ops.act_of(d["x"])
                yp, ya = ops.act_of(y)
                if grouped:
                    cg.add(0, xp, xa, d["w0"], d["b"], yp, ya, Spec(d["k"]), 0.0, st)
                else:
                    _lib.call("vae2_conv2d_fwd", xp, ctypes.byref(xa), ops.ptr(d["w0"]),
                              ops.ptr(d["b"]), yp, ctypes.byref(ya), d["k"], 1, d["k"] // 2,
                              0.0, ops.ptr(st), s)
                outs.append(y)
                stats.append(st)
            if grouped:
                cg.flush()
            shared = None
            for i, d in enumerate(L):
                n, h, w, cin, cout = d["shape"]
                # layers 0 and 4 have the same input shape: both write one dx (beta 0, 1)
                if i == 4:
                    dx, beta = shared, 1.0
                else:
                    dx, beta = ops.new_act((n, h, w, cin), like), 0.0
                    if i == 0:
                        shared = dx
                dyp, dya = ops.act_of(d["dy"])
                dxp, dxa = ops.act_of(dx)
                if grouped:
                    cg.add(1, dyp, dya, d["w1"], None, dxp, dxa, Spec(d["k"]), beta)
                else:
                    _lib.call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dya), ops.ptr(d["w1"]),
                              dxp, ctypes.byref(dxa), d["k"], 1, d["k"] // 2, beta, s)
                dxs.append(dx)
            if grouped:
                cg.flush()
            torch.cuda.synchronize()
            return outs, stats, dxs

        a = run(False)
        lib.vae2_kernel_log(1)
        b = run(True)
        buf = ctypes.create_string_buffer(1 << 14)
        lib.vae2_kernel_log_read(buf, len(buf))
        lib.vae2_kernel_log(0)
        names = buf.value.decode().split(";")
    finally:
        lib.vae2_conv2d_set_algo(prev)
        lib.vae2_conv2d_set_grouping(prev_g)
        lib.vae2_conv2d_set_tune(15, prev_k)
    assert any(nm.startswith("dconv3_group_kernel") for nm in names), names
    assert len(names) < 2 * len(MULTI_SHAPES), names  # fewer launches than jobs
    for ta, tb in zip(a, b):
        for u, v in zip(ta, tb):
            assert torch.equal(u, v)


@pytest.mark.parametrize("hw", [(32, 64), (30, 22), (128, 256)])
def test_up_avgpool_equals_upsample_then_pool(hw):
    """ops.up_avgpool (weighted pooling at the branch resolutions: vae2_weighted_avgpool_*)
    against avgpool(up_cat(xs)) (the materialised full-resolution concatenation), forward
    and backward."""
    from vae2 import ops
    torch.manual_seed(2)
    H, W = hw
    sizes = [(H, W)]
    for _ in range(3):
        sizes.append(((sizes[-1][0] + 1) // 2, (sizes[-1][1] + 1) // 2))
    like = torch.empty(1, device=DEV)
    xs = [ops.new_act((2, h, w, c), like).normal_() for (h, w), c in zip(sizes, (18, 36, 72, 144))]
    g = torch.randn(2, 1, 1, 270, device=DEV)
    outs = []
    for fused in (True, False):
        ops.UP_AVGPOOL = fused
        try:
            leaves = [x.detach().clone().requires_grad_() for x in xs]
            y = ops.up_avgpool(leaves)
            y.backward(g)
            torch.cuda.synchronize()
            outs.append((y.detach(), [t.grad for t in leaves]))
        finally:
            ops.UP_AVGPOOL = True
    (y1, g1), (y0, g0) = outs
    assert rel(y1, y0) < 1e-6
    for a, b in zip(g1, g0):
        assert rel(a, b) < 1e-6


GEMM1_SHAPES = [
    # N, H, W, Cin, Cout, bias: 1x1 convs with >= 65536 pixels through the persistent
    # LDS-weight GEMM (gemm1x1_kernel): the layer-1 expansions / reductions, a padded
    # channel quad (70) with 2 N blocks of 5 tiles, a 3-block N (270)
    (2, 128, 256, 64, 256, False),
    (2, 128, 256, 256, 64, False),
    (1, 256, 256, 70, 130, True),
    (1, 128, 512, 36, 270, True),
]


@pytest.mark.parametrize("tune", [(), ((4, 8), (5, 1))], ids=["default", "tn8-tm1"])
@pytest.mark.parametrize("shape", GEMM1_SHAPES)
def test_gemm1x1(shape, tune):
    """Forward (+ BN statistics through conv_bn), data gradient (+ beta = 1 accumulation
    of a GradLink) and weight gradient against PyTorch fp32 on the CPU; also with the
    8-N-tile, 16-row-tile instances (vae2_conv2d_set_tune keys 4 / 5)."""
    from vae2 import _lib
    lib = _lib.load()
    prev = [(k, lib.vae2_conv2d_set_tune(k, v)) for k, v in tune]
    try:
        _gemm1x1_case(shape)
    finally:
        for k, v in reversed(prev):
            lib.vae2_conv2d_set_tune(k, v)


def _gemm1x1_case(shape):
    from vae2 import ops, prof
    torch.manual_seed(8)
    n, h, w, cin, cout, bias = shape
    conv = nn.Conv2d(cin, cout, 1, 1, 0, bias=bias)
    x = torch.randn(n, cin, h, w, requires_grad=True)
    y_ref = conv(x)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    cg = nn.Conv2d(cin, cout, 1, 1, 0, bias=bias).to(DEV)
    cg.load_state_dict(conv.state_dict())
    xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
    with torch.no_grad():
        xg.copy_(nhwc(x.detach()).to(DEV))
    xg.requires_grad_(True)
    _, xa = ops.act_of(xg)
    assert prof.fwd_kernel_name(xa, (n, h, w, cout), 1, 1, 0).startswith("gemm1x1_kernel")
    dyg = ops.new_act((n, h, w, cout), xg)
    with torch.no_grad():
        dyg.copy_(nhwc(gy).to(DEV))
    yg = ops.conv(xg, cg)
    yg.backward(dyg)
    torch.cuda.synchronize()
    assert rel(nchw(yg), y_ref) < TOL
    assert rel(nchw(xg.grad), x.grad) < TOL
    assert rel(cg.weight.grad, conv.weight.grad) < TOL
    if bias:
        assert rel(cg.bias.grad, conv.bias.grad) < TOL
    # data gradient accumulated onto another consumer's (GradLink, beta = 1)
    link = ops.GradLink(2)
    other = torch.randn(n, h, w, cin)
    link.buf = ops.new_act((n, h, w, cin), xg)
    with torch.no_grad():
        link.buf.copy_(other.to(DEV))
    link.done = 1
    x2 = xg.detach().clone().requires_grad_(True)
    spec = ops.ConvSpec(cg)
    spec.x_link = link
    dx, _, _ = ops._conv_bwd(x2, cg.weight, cg.bias, dyg, spec, True, False, False)
    torch.cuda.synchronize()
    assert rel(dx.cpu(), nhwc(x.grad) + other) < TOL
    # training BatchNorm after the conv: statistics from the persistent kernel's rows
    if not bias:
        bn = nn.BatchNorm2d(cout, momentum=0.01)
        bg = nn.BatchNorm2d(cout, momentum=0.01).to(DEV)
        ref = F.relu(bn(conv(x.detach())))
        out = ops.conv_bn(xg.detach(), cg, bg, relu=True)
        torch.cuda.synchronize()
        assert rel(nchw(out), ref) < TOL
        assert rel(bg.running_mean, bn.running_mean) < 1e-5
        assert rel(bg.running_var, bn.running_var) < 1e-5


@pytest.mark.parametrize("shape", [
    # N, H, W, Cin, Cout, k, stride: gather weight gradients with 16-byte channel-quad
    # operand loads (aligned NHWC: wgrad_kernel<..., V4>), incl. padded quads (18, 5, 7)
    (2, 32, 64, 18, 36, 3, 2),
    (2, 16, 32, 36, 72, 3, 2),
    (2, 64, 64, 64, 64, 1, 1),
    (1, 9, 13, 5, 7, 3, 2),
    (2, 12, 20, 256, 18, 3, 2),
])
def test_wgrad_quad_loads(shape):
    from vae2 import ops
    torch.manual_seed(9)
    n, h, w, cin, cout, k, s = shape
    conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=False)
    x = torch.randn(n, cin, h, w)
    y_ref = conv(x)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    cg = nn.Conv2d(cin, cout, k, s, k // 2, bias=False).to(DEV)
    cg.load_state_dict(conv.state_dict())
    xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
    with torch.no_grad():
        xg.copy_(nhwc(x).to(DEV))
    oh, ow = y_ref.shape[2:]
    dyg = ops.new_act((n, oh, ow, cout), xg)
    with torch.no_grad():
        dyg.copy_(nhwc(gy).to(DEV))
    spec = ops.ConvSpec(cg)
    _, wret, _ = ops._conv_bwd(xg, cg.weight, None, dyg, spec, False, True, False)
    ops.flush_wgrad()
    torch.cuda.synchronize()
    got = cg.weight.grad if wret is None else wret
    assert rel(got, conv.weight.grad) < TOL
