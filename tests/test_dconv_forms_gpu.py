"""Two launch forms of the direct 3x3 conv for layers short of workgroups (the W18 72-channel
branch at 32 x 64: 256 workgroups, one wave per SIMD; enc_hrnet.py:27-62):
  split72 (vae2_conv2d_set_tune key 14): 72 channels as two N blocks of 32 MFMA + 4 VALU
          channels instead of two padded 48-column blocks;
  ksp     (key 15 = 1): the same 4-row tiles as 8-wave workgroups splitting K in two (K chunk
          pairs alternate between the wave sets, summed through LDS in a fixed order);
  ksp4    (key 15 = 2): 16-wave workgroups, K in four shares.
Each against fp64 PyTorch and against the default form: forward (+ bias, + beta * y, BN
partial statistics), forward with the producer BatchNorm applied in the staging, data
gradient (+ beta) and the data gradient's producer-BatchNorm backward partials.  Shapes: the
bench layer, a partial strip with H % 4 = 1, a padded input quad, and (ksp) 64 / 32 channels
(4 / 2 column tiles)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from test_dconv_stream_gpu import _bn_save, _fwd, _names, _nchw, _nhwc, rel, sums_ok

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [
    # N, H, W, Cin, Cout (auto dispatch: the direct kernel, 256-511 workgroups)
    (8, 32, 64, 72, 72),   # the bench layer
    (6, 29, 80, 72, 72),   # partial strip, H % 4 = 1
    (6, 32, 72, 70, 72),   # padded input channel quad
    (8, 32, 128, 64, 64),  # ksp only: one N block of 4 tiles
    (8, 32, 128, 32, 32),  # ksp only: 2 tiles
]
KEY = {"split72": (14, 1), "ksp": (15, 1), "ksp4": (15, 2)}


def _lib():
    from vae2 import _lib
    return _lib.load()


@pytest.fixture(params=["split72", "ksp", "ksp4"])
def form(request):
    lib = _lib()
    prev = lib.vae2_conv2d_set_algo(0)
    prevs = {k: lib.vae2_conv2d_set_tune(k, 0) for k in (14, 15)}
    lib.vae2_conv2d_set_tune(*KEY[request.param])
    yield request.param
    for k, v in prevs.items():
        lib.vae2_conv2d_set_tune(k, v)
    lib.vae2_conv2d_set_algo(prev)


def _switch(form, on):
    key, val = KEY[form]
    _lib().vae2_conv2d_set_tune(key, val if on else 0)


def _skip(form, shape):
    if form == "split72" and shape[4] != 72:
        pytest.skip("72 output channels only")


def _args(names, flip):
    """Template arguments of the one dconv3 instance of the direction."""
    tag = "true" if flip else "false"
    args = [[s.strip() for s in k[len("dconv3_kernel<"):k.index(">")].split(",")]
            for k in names if k.startswith("dconv3_kernel<")]
    args = [a for a in args if a[2] == tag]
    assert len(args) == 1, names
    return args[0]


def _check(form, names, flip, on=True):
    a = _args(names, flip)
    if form == "split72":
        assert (int(a[1]), int(a[4])) == ((2, 4) if on else (3, 0)), a
    else:
        ks = (2 if form == "ksp" else 4) if on else 1
        assert a[6:8] == [str(4 * ks), str(ks)] and int(a[4]) == 0, a


@pytest.mark.parametrize("shape", SHAPES)
def test_form_forward_stats(form, shape):
    _skip(form, shape)
    torch.manual_seed(21)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    bias = torch.randn(cout, device=DEV)
    xg = _nhwc(x)
    ref = F.conv2d(x.double(), wt.double(), bias.double(), 1, 1)
    outs = {}
    for on in (True, False):
        _switch(form, on)
        y, st, names = _fwd(xg, wt, bias, stats_rows=True)
        _check(form, names, False, on)
        assert rel(_nchw(y), ref) < 1e-6
        assert torch.isfinite(st).all()  # every statistics row written
        sums = st.double().sum(1)
        assert sums_ok(sums[0], ref) and sums_ok(sums[1], ref * ref)
        outs[on] = (y.clone(), st.shape)
    assert rel(outs[True][0], outs[False][0]) < 1e-6
    assert outs[True][1] == outs[False][1]  # the same partial-statistics rows


@pytest.mark.parametrize("shape", SHAPES[:2] + SHAPES[4:])
def test_form_forward_beta(form, shape):
    _skip(form, shape)
    torch.manual_seed(22)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    old = torch.randn(n, cout, h, w, device=DEV)
    ref = F.conv2d(x.double(), wt.double(), None, 1, 1) + 0.5 * old.double()
    y, st, names = _fwd(_nhwc(x), wt, None, y=_nhwc(old), beta=0.5, stats_rows=True)
    _check(form, names, False)
    assert rel(_nchw(y), ref) < 1e-6
    sums = st.double().sum(1)
    assert sums_ok(sums[0], ref) and sums_ok(sums[1], ref * ref)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("relu", [0, 1])
def test_form_forward_input_bn(form, shape, relu):
    _skip(form, shape)
    torch.manual_seed(23)
    n, h, w, cin, cout = shape
    x = torch.randn(n, cin, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    sv = _bn_save(cin, 5)
    xb = x.double() * sv[2].double().view(1, -1, 1, 1) + sv[3].double().view(1, -1, 1, 1)
    if relu:
        xb = xb.clamp_min(0)
    ref = F.conv2d(xb, wt.double(), None, 1, 1)
    y, st, names = _fwd(_nhwc(x), wt, None, stats_rows=True, bn_save=sv, relu=relu)
    _check(form, names, False)
    assert rel(_nchw(y), ref) < 1e-6
    assert sums_ok(st.double().sum(1)[0], ref)


SQUARE = [s for s in SHAPES if s[3] == s[4]]


@pytest.mark.parametrize("shape", SQUARE)
def test_form_data_gradient(form, shape):
    _skip(form, shape)
    from vae2 import ops
    torch.manual_seed(24)
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
    _check(form, names, True)
    assert rel(_nchw(dx), ref) < 1e-6
    run(1.0)
    torch.cuda.synchronize()
    assert rel(_nchw(dx), 2 * ref) < 1e-6


@pytest.mark.parametrize("shape", SQUARE)
@pytest.mark.parametrize("relu", [0, 1])
def test_form_data_gradient_bn_partials(form, shape, relu):
    _skip(form, shape)
    from vae2 import ops
    torch.manual_seed(25)
    n, h, w, cin, cout = shape
    dy = torch.randn(n, cout, h, w, device=DEV)
    wt = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    bx = torch.randn(n, cin, h, w, device=DEV)
    sv = _bn_save(cin, 6)
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
    _check(form, names, True)
    assert rel(_nchw(dx), dxr) < 1e-6
    assert torch.isfinite(part).all()
    sums = part.double().sum(1)
    assert sums_ok(sums[0], g) and sums_ok(sums[1], g * xhat)
