"""The streaming direct 3x3 kernel (csrc/dconv_stream.hip: 18 -> 18 and 36 -> 36 channels,
bands of a 32-column strip walked 4 output rows per step through an LDS ring) against
fp64 PyTorch and against the per-tile kernel it replaces (vae2_conv2d_set_tune key 9 = 0):
forward (+ bias, + beta * y, BN partial statistics, unaligned / unpadded outputs), forward
with the producer BatchNorm applied in the staging, data gradient (+ beta) and the data
gradient's producer-BatchNorm backward partials.  Shapes cover partial strips, heights
that are not a multiple of 4, single-step bands, several bands per strip and the padded
channel quad (17 input channels)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [
    # N, H, W, Cin, Cout
    (2, 16, 32, 18, 18),
    (2, 13, 40, 18, 18),    # partial strip (8 columns), H % 4 = 1
    (1, 5, 20, 18, 18),     # one partial strip, 2 steps
    (2, 9, 33, 17, 18),     # padded channel quad, 1-column strip
    (8, 128, 256, 18, 18),  # the 128 x 256 branch: several bands per strip
    (2, 16, 32, 36, 36),
    (2, 11, 70, 36, 36),
    (8, 64, 128, 36, 36),   # the 64 x 128 branch
]


def _lib():
    from vae2 import _lib
    return _lib.load()


def _names(fn):
    from test_bench_instances_gpu import Recorder
    with Recorder() as rec:
        out = fn()
        torch.cuda.synchronize()
    return out, [k for _, _, ks in rec.calls for k in ks]


def _nhwc(t, pad4=True):
    from vae2 import ops
    n, c, h, w = t.shape
    a = ops.new_act((n, h, w, c), t) if pad4 else torch.empty((n, h, w, c), device=t.device)
    with torch.no_grad():
        a.copy_(t.permute(0, 2, 3, 1))
    return a


def _nchw(a):
    return a.permute(0, 3, 1, 2)


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def sums_ok(got, terms, tol=2e-6):
    """Per-channel sums against fp64, relative to the sum of magnitudes (zero-mean terms
    leave the sum itself near zero)."""
    err = (got.double() - terms.sum((0, 2, 3))).abs()
    return (err / terms.abs().sum((0, 2, 3)).clamp_min(1e-30)).max().item() < tol


def _stream(on):
    return _lib().vae2_conv2d_set_tune(9, 3 if on else 0)


def _fwd(x, w, bias=None, y=None, beta=0.0, stats_rows=False, bn_save=None, relu=0):
    """vae2_conv2d_fwd / _fwd_bnin through the C ABI; returns (y, stats or None, names)."""
    from vae2 import ops
    lib = _lib()
    xp, xa = ops.act_of(x)
    cout = w.shape[0]
    if y is None:
        y = ops.new_act((x.shape[0], x.shape[1], x.shape[2], cout), x)
        y.zero_()
    yp, ya = ops.act_of(y)
    stats = None
    if stats_rows:
        rows = lib.vae2_conv2d_fwd_stats_rows(xp, ctypes.byref(xa), ctypes.byref(ya), 3, 1, 1)
        assert rows > 0
        stats = torch.full((2, rows, cout), float("nan"), device=DEV)
    wp = ops.packed_weight(w, 0)
    s = ops.stream_ptr()

    def run():
        if bn_save is not None:
            ops.call("vae2_conv2d_fwd_bnin", xp, ctypes.byref(xa), ops.ptr(bn_save), relu,
                     ops.ptr(wp), ops.ptr(bias), yp, ctypes.byref(ya), 3, 1, 1, beta,
                     ops.ptr(stats), s)
        else:
            ops.call("vae2_conv2d_fwd", xp, ctypes.byref(xa), ops.ptr(wp), ops.ptr(bias), yp,
                     ctypes.byref(ya), 3, 1, 1, beta, ops.ptr(stats), s)
    _, names = _names(run)
    return y, stats, names


def _bn_save(c, seed):
    g = torch.Generator().manual_seed(seed)
    mean = torch.randn(c, generator=g) * 0.3
    invstd = 1.0 / (torch.rand(c, generator=g) + 0.5)
    gamma = torch.randn(c, generator=g) * 0.5 + 1.0
    beta = torch.randn(c, generator=g) * 0.3
    scale = gamma * invstd
    shift = beta - mean * scale
    return torch.stack([mean, invstd, scale, shift]).float().to(DEV).contiguous()


def _check_names(names, flip):
    tag = "true" if flip else "false"
    assert any(k.startswith("dconv3s_kernel") and f", {tag}, " in k for k in names), names


@pytest.fixture(autouse=True)
def _algo():
    lib = _lib()
    prev = lib.vae2_conv2d_set_algo(2)
    prev_s = lib.vae2_conv2d_set_tune(9, 3)  # 18 and 36 channels
    yield
    lib.vae2_conv2d_set_tune(9, prev_s)
    lib.vae2_conv2d_set_algo(prev)


@pytest.mark.parametrize("shape", SHAPES)
def test_stream_forward_stats(shape):
    torch.manual_seed(11)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    bias = torch.randn(cout, device=DEV)
    xg = _nhwc(x)
    y, st, names = _fwd(xg, wt, bias, stats_rows=True)
    _check_names(names, False)
    ref = F.conv2d(x.double(), wt.double(), bias.double(), 1, 1)
    assert rel(_nchw(y), ref) < 1e-6
    sums = st.double().sum(1)
    assert sums_ok(sums[0], ref) and sums_ok(sums[1], ref * ref)
    # the per-tile kernel: same conv up to fp32 summation order
    _stream(False)
    y0, st0, names0 = _fwd(xg, wt, bias, stats_rows=True)
    assert not any(k.startswith("dconv3s_kernel") for k in names0)
    assert rel(y, y0) < 1e-6
    assert sums_ok(sums[0] - st0.double().sum(1)[0] + ref.sum((0, 2, 3)), ref)


@pytest.mark.parametrize("shape", [SHAPES[1], SHAPES[3], SHAPES[6]])
def test_stream_forward_beta_and_unpadded_output(shape):
    """beta * y accumulation (loads of the old output in the MFMA layout) with statistics of
    the stored sum, into a 16-byte aligned padded output and into an unpadded NHWC one
    (pixel stride 18 / 36: the element-store path)."""
    torch.manual_seed(12)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    old = torch.randn(n, cout, h, w, device=DEV)
    ref = F.conv2d(x.double(), wt.double(), None, 1, 1) + 0.5 * old.double()
    xg = _nhwc(x)
    for pad4 in (True, False):
        y, st, names = _fwd(xg, wt, None, y=_nhwc(old, pad4), beta=0.5, stats_rows=True)
        _check_names(names, False)
        assert rel(_nchw(y), ref) < 1e-6
        sums = st.double().sum(1)
        assert sums_ok(sums[0], ref) and sums_ok(sums[1], ref * ref)


@pytest.mark.parametrize("shape", [SHAPES[0], SHAPES[1], SHAPES[4], SHAPES[6]])
@pytest.mark.parametrize("relu", [0, 1])
def test_stream_forward_input_bn(shape, relu):
    """relu?(x * scale + shift) applied in the staging: in-image pixels only (the zero halo
    of the padded conv stays zero), padded channel quad zero."""
    torch.manual_seed(13)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    sv = _bn_save(cin, 3)
    xb = x.double() * sv[2].double().view(1, -1, 1, 1) + sv[3].double().view(1, -1, 1, 1)
    if relu:
        xb = xb.clamp_min(0)
    ref = F.conv2d(xb, wt.double(), None, 1, 1)
    y, st, names = _fwd(_nhwc(x), wt, None, stats_rows=True, bn_save=sv, relu=relu)
    _check_names(names, False)
    assert rel(_nchw(y), ref) < 1e-6
    assert sums_ok(st.double().sum(1)[0], ref)


SQUARE = [s for s in SHAPES if s[3] == s[4]]  # the data gradient's output is the forward input


@pytest.mark.parametrize("shape", SQUARE)
def test_stream_data_gradient(shape):
    """dx = conv_transpose(dy) (flipped taps, mode-1 weights), overwrite then beta = 1
    accumulation (a GradLink's second consumer)."""
    from vae2 import ops
    torch.manual_seed(14)
    n, h, w, cin, cout = shape
    dy = torch.randn(n, cout, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.double(), dy.double(), 1, 1)
    dyg = _nhwc(dy)
    dx = ops.new_act((n, h, w, cin), dyg)
    dyp, dya = ops.act_of(dyg)
    dxp, dxa = ops.act_of(dx)
    wp = ops.packed_weight(wt, 1)

    def run(beta):
        ops.call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dya), ops.ptr(wp), dxp,
                 ctypes.byref(dxa), 3, 1, 1, beta, ops.stream_ptr())
    _, names = _names(lambda: run(0.0))
    _check_names(names, True)
    assert rel(_nchw(dx), ref) < 1e-6
    run(1.0)
    torch.cuda.synchronize()
    assert rel(_nchw(dx), 2 * ref) < 1e-6


@pytest.mark.parametrize("shape", [SHAPES[0], SHAPES[1], SHAPES[2], SHAPES[4], SHAPES[7]])
@pytest.mark.parametrize("relu", [0, 1])
def test_stream_data_gradient_bn_partials(shape, relu):
    """The producer BatchNorm's backward partials from the data-gradient epilogue: rows sum
    to (sum g, sum g * xhat) with g = dx masked by the producer's ReLU."""
    from vae2 import ops
    torch.manual_seed(15)
    n, h, w, cin, cout = shape
    dy = torch.randn(n, cout, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    bx = torch.randn(n, cin, h, w, device=DEV)
    sv = _bn_save(cin, 4)
    dxr = torch.nn.grad.conv2d_input((n, cin, h, w), wt.double(), dy.double(), 1, 1)
    sc, sh = sv[2].double().view(1, -1, 1, 1), sv[3].double().view(1, -1, 1, 1)
    g = dxr * ((bx.double() * sc + sh) > 0) if relu else dxr
    xhat = (bx.double() - sv[0].double().view(1, -1, 1, 1)) * sv[1].double().view(1, -1, 1, 1)
    dyg, bxg = _nhwc(dy), _nhwc(bx)
    dx = ops.new_act((n, h, w, cin), dyg)
    dyp, dya = ops.act_of(dyg)
    dxp, dxa = ops.act_of(dx)
    bxp, bxa = ops.act_of(bxg)
    rows = _lib().vae2_conv2d_bwd_data_bnpart_rows(dyp, ctypes.byref(dya), ctypes.byref(dxa), 3, 1, 1)
    assert rows > 0
    part = torch.full((2, rows, cin), float("nan"), device=DEV)
    wp = ops.packed_weight(wt, 1)
    _, names = _names(lambda: ops.call(
        "vae2_conv2d_bwd_data_bnpart", dyp, ctypes.byref(dya), ops.ptr(wp), dxp,
        ctypes.byref(dxa), 3, 1, 1, bxp, ctypes.byref(bxa), ops.ptr(sv), relu, ops.ptr(part),
        ops.stream_ptr()))
    _check_names(names, True)
    assert rel(_nchw(dx), dxr) < 1e-6
    sums = part.double().sum(1)
    assert sums_ok(sums[0], g) and sums_ok(sums[1], g * xhat)


def test_stream_rows_match_launch_plan():
    """The statistics rows reported for a shape are what the kernel writes: every row of a
    NaN-filled buffer is overwritten (no row left, none written past the end)."""
    from vae2 import ops
    for shape in SHAPES:
        n, h, w, cin, cout = shape
        x = torch.randn(n, cin, h, w, device=DEV)
        wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
        _, st, _ = _fwd(_nhwc(x), wt, None, stats_rows=True)
        assert torch.isfinite(st).all(), shape
    # the query follows set_tune key 9: bands of the streaming plan (2 x 2 strips x 2 bands
    # of 8 rows at key 17 = 2: at least 2 steps per band; 4 bands of 4 rows at the default 1)
    # vs the per-tile kernel's 4-row tiles (2 x 4 x 2)
    xa = ops.Act(2, 13, 40, 18, 20)
    ya = ops.Act(2, 13, 40, 18, 18)
    lib = _lib()
    rows = lambda: lib.vae2_conv2d_fwd_stats_rows(ctypes.c_void_p(256), ctypes.byref(xa),
                                                  ctypes.byref(ya), 3, 1, 1)
    prev = lib.vae2_conv2d_set_tune(17, 2)
    try:
        r2 = rows()
        lib.vae2_conv2d_set_tune(17, 1)
        r1 = rows()
    finally:
        lib.vae2_conv2d_set_tune(17, prev)
    _stream(False)
    r0 = rows()
    assert (r2, r1, r0) == (8, 16, 16)


@pytest.mark.parametrize("shape", [SHAPES[1], SHAPES[4]])
def test_stream_weight_operand_from_lds_or_global(shape):
    """18 channels: the B operand staged in LDS (set_tune key 11 = 1) or loaded from the
    packed weights (0) -- the same fragments in the same order, so bit-identical outputs and
    statistics."""
    torch.manual_seed(16)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    xg = _nhwc(x)
    lib = _lib()
    outs = []
    prev = lib.vae2_conv2d_set_tune(11, 1)
    try:
        for bl in (1, 0):
            lib.vae2_conv2d_set_tune(11, bl)
            y, st, names = _fwd(xg, wt, None, stats_rows=True)
            _check_names(names, False)
            outs.append((y.clone(), st.clone()))
    finally:
        lib.vae2_conv2d_set_tune(11, prev)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
