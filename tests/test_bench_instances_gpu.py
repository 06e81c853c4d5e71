"""Parity of every kernel instance the benchmark's training step launches, at the exact
geometry it launches them with (BASELINE config 3: HRNet-W18-small-v2, 128x256, B=8).

Tile shape, K split, stride-parity classes, slab widths and the split counts of the
reductions are chosen from M = N*H*W, the channel counts and the pixel strides, so the
kernel instances (and grids) the bench times differ from the ones the small-geometry
parity tests reach.  The full-step backward at this size is too slow for the fp64 CPU
oracle on the test box (~4 min, ~55 GB), so instead:

  * one bench-geometry training step is recorded: every conv call of the C ABI (forward,
    data gradient, weight gradient, the deferred weight-gradient reductions) with its
    exact descriptors (shape, pixel stride, alignment, stride, beta, bias / statistics
    epilogue) and the kernels it launched;
  * every distinct call is replayed on fresh random buffers of that exact layout (pad
    channels filled with garbage) and held to torch-CPU fp32 (F.conv2d and its two
    gradients): rel-L2 2e-5 forward / data gradient, 1e-4 weight gradient (a sum over
    262,144 pixels per element in both implementations), BN partial statistics 1e-5;
  * the heads (270-channel per-branch head path) and a stage-4 HighResolutionModule
    (lock-stepped BatchNorm launches, fuse sums, power-of-two upsample adjoints) run at
    the bench's branch shapes against the reference formulation on CPU;
  * coverage: every conv / BatchNorm / head / fuse kernel instance the step launched was
    launched by these checks.
"""
import copy
import ctypes
import zlib

import pytest
import torch
import torch.nn.functional as F
from torch.nn.grad import conv2d_input, conv2d_weight

from helpers import build, make_cfg, max_rel, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, H, W = 8, 128, 256
CONV_ABI = ("vae2_conv2d_fwd", "vae2_conv2d_bwd_data", "vae2_conv2d_bwd_weight",
            "vae2_conv2d_bwd_weight_ld", "vae2_conv2d_multi", "vae2_wgrad_flush",
            # BatchNorm fused into the consumer conv (ops.LazyBN: dconv3 / wgrad3 BNX = 1, 2)
            "vae2_conv2d_fwd_bnin", "vae2_conv2d_bwd_weight_bnin", "vae2_conv2d_bwd_data_bnpart")
HEAD_ABI = ("vae2_conv1x1_upsum_fwd", "vae2_head_out_fwd", "vae2_head_out_bwd_reduce",
            "vae2_head_out_bwd_apply", "vae2_upsample_bilinear_bwd_multi",
            "vae2_bn_reduce_finalize_shifted")
BN_FUSE_ABI = ("vae2_bn_multi_apply", "vae2_bn_multi_bwd_reduce", "vae2_bn_multi_bwd_apply",
               "vae2_bn_multi_reduce", "vae2_bn_multi_finalize", "vae2_fuse_sum_relu",
               "vae2_relu_bwd", "vae2_relu_bwd_dual", "vae2_upsample_bilinear_bwd_pow2",
               "vae2_upsample_bilinear_bwd", "vae2_upsample_bilinear_fwd")


class Recorder:
    """_lib.CALL_HOOK: each C-ABI call with copied descriptors and its launched kernels."""

    def __init__(self):
        from vae2 import _lib
        self.lib = _lib.load()
        self.buf = ctypes.create_string_buffer(1 << 16)
        self.calls = []

    def __call__(self, name, fn, args):
        self.lib.vae2_kernel_log_read(None, 0)
        desc = describe(name, args)
        rc = fn(*args)
        n = self.lib.vae2_kernel_log_read(self.buf, len(self.buf))
        ks = self.buf.value.decode().split(";") if n > 0 else []
        if desc and desc[0][0] in ("wgrad", "wgrad_bnin"):  # reduction deferred to vae2_wgrad_flush or not
            desc = [d + (not any(k.startswith("wgrad_reduce_kernel") for k in ks),) for d in desc]
        self.calls.append((name, desc, ks))
        return rc

    def __enter__(self):
        from vae2 import _lib
        self.lib.vae2_kernel_log(1)
        _lib.CALL_HOOK = self
        return self

    def __exit__(self, *exc):
        from vae2 import _lib
        _lib.CALL_HOOK = None
        self.lib.vae2_kernel_log(0)


def _act(a):
    o = a._obj if hasattr(a, "_obj") else a
    return (int(o.n), int(o.h), int(o.w), int(o.c), int(o.ps))


def _al(p):
    v = p.value if isinstance(p, ctypes.c_void_p) else p
    return None if v is None else int(v) % 16 // 4  # float offset inside a 16-byte line


def describe(name, args):
    """Hashable replay key(s) of a conv call: list of (kind, ...) tuples."""
    if name == "vae2_conv2d_fwd":
        xp, xa, wp, bias, yp, ya, k, s, pad, beta, stats, _ = args
        return [("fwd", _act(xa), _al(xp), _act(ya), _al(yp), k, s, pad, float(beta) != 0.0,
                 bias is not None and _al(bias) is not None, stats is not None and
                 _al(stats) is not None)]
    if name == "vae2_conv2d_bwd_data":
        dyp, dya, wp, dxp, dxa, k, s, pad, beta, _ = args
        return [("dgrad", _act(dya), _al(dyp), _act(dxa), _al(dxp), k, s, pad,
                 float(beta) != 0.0)]
    if name in ("vae2_conv2d_bwd_weight", "vae2_conv2d_bwd_weight_ld"):
        if name == "vae2_conv2d_bwd_weight":
            xp, xa, dyp, dya, dw, db, k, s, pad, acc = args[:10]
        else:
            xp, xa, dyp, dya, dw, _ld, db, k, s, pad, acc = args[:11]
        return [("wgrad", _act(xa), _al(xp), _act(dya), _al(dyp), k, s, pad, int(acc),
                 db is not None and _al(db) is not None)]
    if name == "vae2_conv2d_fwd_bnin":
        xp, xa, _save, relu, wp, bias, yp, ya, k, s, pad, beta, stats, _ = args
        return [("fwd_bnin", _act(xa), _al(xp), _act(ya), _al(yp), k, s, pad,
                 float(beta) != 0.0, bias is not None and _al(bias) is not None,
                 stats is not None and _al(stats) is not None, int(relu))]
    if name == "vae2_conv2d_bwd_weight_bnin":
        xp, xa, _save, relu, dyp, dya, dw, db, k, s, pad, acc = args[:12]
        return [("wgrad_bnin", _act(xa), _al(xp), _act(dya), _al(dyp), k, s, pad, int(acc),
                 db is not None and _al(db) is not None, int(relu))]
    if name == "vae2_conv2d_bwd_data_bnpart":
        dyp, dya, wp, dxp, dxa, k, s, pad, bxp, bxa, _save, relu, _part, _ = args
        return [("dgrad_bnpart", _act(dya), _al(dyp), _act(dxa), _al(dxp), k, s, pad,
                 _act(bxa), _al(bxp), int(relu))]
    if name == "vae2_conv2d_multi":
        n, arr, _ = args
        jobs = ctypes.cast(arr, ctypes.POINTER(_job_type()))
        out = []
        for i in range(int(n)):
            j = jobs[i]
            if j.kind == 0:
                out.append(("fwd", _act(j.xd), _al(j.x), _act(j.yd), _al(j.y), j.k, j.stride,
                            j.pad, float(j.beta) != 0.0, bool(j.bias), bool(j.stats)))
            else:
                out.append(("dgrad", _act(j.xd), _al(j.x), _act(j.yd), _al(j.y), j.k, j.stride,
                            j.pad, float(j.beta) != 0.0))
        return out
    return None


def _job_type():
    from vae2 import _lib
    return _lib.ConvJob


@pytest.fixture(scope="module")
def bench_step():
    """One eager training step of the bench's model at the bench's geometry, recorded."""
    from vae2.model import FullModel_encdec
    from vae2.optim import FusedAdam
    ed, ez = build(make_cfg(arch="w18", hw=(H, W)))
    fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(DEV)
    fm.train()
    opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-4)
    gen = torch.Generator().manual_seed(9)
    xs = [torch.randn(B, 9, H, W, generator=gen).to(DEV) for _ in range(3)]
    fm.set_noise(torch.randn(B, 10, 1, 1, generator=gen), torch.randn(B, 10, 1, 1, generator=gen))
    with Recorder() as rec:
        opt.zero_grad()
        losses = fm(*xs, 1.0)[0]
        losses[0].backward()
        opt.step()
        torch.cuda.synchronize()
    assert torch.isfinite(losses[0]).all()
    return rec.calls


def _family(kernel):
    from vae2 import prof
    return prof.family(kernel)


def _buffer(act, align, fill=True):
    """Device buffer laid out like the recorded descriptor: (data view (n,h,w,c), base).
    Pixel-stride padding channels hold garbage the kernels must ignore."""
    n, h, w, c, ps = act
    off = align or 0
    base = torch.randn(n * h * w * ps + off + 8, device=DEV) if fill else \
        torch.empty(n * h * w * ps + off + 8, device=DEV)
    view = base[off:off + n * h * w * ps].view(n, h, w, ps)[..., :c]
    return view, base


def _nchw(v):
    return v.permute(0, 3, 1, 2).detach().cpu()


def _replay_fwd(key, lib):
    from vae2 import ops
    _, xa, xal, ya, yal, k, s, pad, beta, has_bias, has_stats = key
    x, _ = _buffer(xa, xal)
    y, _ = _buffer(ya, yal)
    y0 = y.clone()
    cout, cin = ya[3], xa[3]
    g = torch.Generator().manual_seed(zlib.crc32(repr(key).encode()))
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(DEV)
    b = (0.1 * torch.randn(cout, generator=g)).to(DEV) if has_bias else None
    xp, xact = ops.act_of(x)
    yp, yact = ops.act_of(y)
    stats, rows = None, 0
    if has_stats:
        rows = lib.vae2_conv2d_fwd_stats_rows(xp, ctypes.byref(xact), ctypes.byref(yact), k, s,
                                              pad)
        stats = torch.empty(2 * rows * cout, device=DEV)
    ops.call("vae2_conv2d_fwd", xp, ctypes.byref(xact), ops.ptr(ops.packed_weight(w, 0)),
             ops.ptr(b), yp, ctypes.byref(yact), k, s, pad, 1.0 if beta else 0.0, ops.ptr(stats),
             ops.stream_ptr())
    torch.cuda.synchronize()
    ref = F.conv2d(_nchw(x), w.cpu(), b.cpu() if b is not None else None, s, pad)
    if beta:
        ref = ref + _nchw(y0)
    got = _nchw(y)
    assert rel(got, ref) < 2e-5, (key, rel(got, ref))
    if has_stats:
        st = stats.view(2, rows, cout).double().sum(1).cpu()
        want = torch.stack([got.double().sum((0, 2, 3)), (got.double() ** 2).sum((0, 2, 3))])
        assert rel(st, want) < 1e-5, (key, rel(st, want))


def _replay_dgrad(key, lib):
    from vae2 import ops
    _, dya, dyal, dxa, dxal, k, s, pad, beta = key
    dy, _ = _buffer(dya, dyal)
    dx, _ = _buffer(dxa, dxal)
    dx0 = dx.clone()
    cout, cin = dya[3], dxa[3]
    g = torch.Generator().manual_seed(zlib.crc32(repr(key).encode()))
    w = (torch.randn(cout, cin, k, k, generator=g) / (cout * k * k) ** 0.5).to(DEV)
    dyp, dyact = ops.act_of(dy)
    dxp, dxact = ops.act_of(dx)
    ops.call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dyact), ops.ptr(ops.packed_weight(w, 1)),
             dxp, ctypes.byref(dxact), k, s, pad, 1.0 if beta else 0.0, ops.stream_ptr())
    torch.cuda.synchronize()
    n, h, wd, _, _ = dxa
    ref = conv2d_input((n, cin, h, wd), w.cpu(), _nchw(dy), s, pad)
    if beta:
        ref = ref + _nchw(dx0)
    assert rel(_nchw(dx), ref) < 2e-5, (key, rel(_nchw(dx), ref))


def _replay_wgrad(key, lib):
    """With the slab reduction deferred (vae2_wgrad_defer + flush) or not, as in the step."""
    from vae2 import ops
    _, xa, xal, dya, dyal, k, s, pad, acc, has_bias, deferred = key
    x, _ = _buffer(xa, xal)
    dy, _ = _buffer(dya, dyal)
    cout, cin = dya[3], xa[3]
    dw = torch.randn(cout, cin, k, k, device=DEV)
    dw0 = dw.clone()
    db = torch.randn(cout, device=DEV) if has_bias else None
    db0 = db.clone() if has_bias else None
    xp, xact = ops.act_of(x)
    dyp, dyact = ops.act_of(dy)
    size = lib.vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xact), ctypes.byref(dyact), k)
    ws = torch.empty(max(size, 1), device=DEV)
    lib.vae2_wgrad_defer(1 if deferred else 0)
    try:
        ops.call("vae2_conv2d_bwd_weight", xp, ctypes.byref(xact), dyp, ctypes.byref(dyact),
                 ops.ptr(dw), ops.ptr(db), k, s, pad, acc, ops.ptr(ws), size, ops.stream_ptr())
        if deferred:
            ops.call("vae2_wgrad_flush", ops.stream_ptr())
    finally:
        lib.vae2_wgrad_defer(0)
    torch.cuda.synchronize()
    ref = conv2d_weight(_nchw(x), (cout, cin, k, k), _nchw(dy), s, pad)
    if acc:
        ref = ref + dw0.cpu()
    assert rel(dw.cpu(), ref) < 1e-4, (key, rel(dw.cpu(), ref))
    if has_bias:
        rb = _nchw(dy).sum((0, 2, 3)) + (db0.cpu() if acc else 0.0)
        assert rel(db.cpu(), rb) < 1e-5, (key, rel(db.cpu(), rb))


def _bn_save(c, g, relu_frac=0.5):
    """A BatchNorm layer's (mean, invstd, scale, shift) with some channels' shift making
    the ReLU cut a good share of the pixels (random, not the reference init's ~identity)."""
    mean = 0.3 * torch.randn(c, generator=g)
    invstd = 0.5 + torch.rand(c, generator=g)
    gamma = 1.0 + 0.5 * torch.randn(c, generator=g)
    beta = relu_frac * torch.randn(c, generator=g)
    scale = gamma * invstd
    return torch.cat([mean, invstd, scale, beta - mean * scale]).contiguous()


def _normalised(x, save, relu):
    """The stored path's input: relu?(x * scale + shift) on CPU (NCHW)."""
    c = x.shape[1]
    z = x * save[2 * c:3 * c].view(1, c, 1, 1) + save[3 * c:].view(1, c, 1, 1)
    return z.clamp_min(0.0) if relu else z


def _replay_fwd_bnin(key, lib):
    """conv(relu(bn(r))) with bn applied while staging r, vs normalise-then-conv on CPU."""
    from vae2 import ops
    _, xa, xal, ya, yal, k, s, pad, beta, has_bias, has_stats, relu = key
    x, _ = _buffer(xa, xal)
    y, _ = _buffer(ya, yal)
    y0 = y.clone()
    cout, cin = ya[3], xa[3]
    g = torch.Generator().manual_seed(zlib.crc32(repr(key).encode()))
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(DEV)
    b = (0.1 * torch.randn(cout, generator=g)).to(DEV) if has_bias else None
    save = _bn_save(cin, g)
    save_d = save.to(DEV)
    xp, xact = ops.act_of(x)
    yp, yact = ops.act_of(y)
    stats, rows = None, 0
    if has_stats:
        rows = lib.vae2_conv2d_fwd_stats_rows(xp, ctypes.byref(xact), ctypes.byref(yact), k, s,
                                              pad)
        stats = torch.empty(2 * rows * cout, device=DEV)
    ops.call("vae2_conv2d_fwd_bnin", xp, ctypes.byref(xact), ops.ptr(save_d), relu,
             ops.ptr(ops.packed_weight(w, 0)), ops.ptr(b), yp, ctypes.byref(yact), k, s, pad,
             1.0 if beta else 0.0, ops.ptr(stats), ops.stream_ptr())
    torch.cuda.synchronize()
    z = _normalised(_nchw(x), save, relu)
    ref = F.conv2d(z, w.cpu(), b.cpu() if b is not None else None, s, pad)
    if beta:
        ref = ref + _nchw(y0)
    got = _nchw(y)
    assert rel(got, ref) < 2e-5, (key, rel(got, ref))
    if has_stats:
        st = stats.view(2, rows, cout).double().sum(1).cpu()
        want = torch.stack([got.double().sum((0, 2, 3)), (got.double() ** 2).sum((0, 2, 3))])
        assert rel(st, want) < 1e-5, (key, rel(st, want))


def _replay_wgrad_bnin(key, lib):
    """dW of conv(relu(bn(r))) with bn applied to the staged r, vs CPU fp32."""
    from vae2 import ops
    _, xa, xal, dya, dyal, k, s, pad, acc, has_bias, relu, deferred = key
    x, _ = _buffer(xa, xal)
    dy, _ = _buffer(dya, dyal)
    cout, cin = dya[3], xa[3]
    g = torch.Generator().manual_seed(zlib.crc32(repr(key).encode()))
    save = _bn_save(cin, g)
    save_d = save.to(DEV)
    dw = torch.randn(cout, cin, k, k, device=DEV)
    dw0 = dw.clone()
    db = torch.randn(cout, device=DEV) if has_bias else None
    xp, xact = ops.act_of(x)
    dyp, dyact = ops.act_of(dy)
    size = lib.vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xact), ctypes.byref(dyact), k)
    ws = torch.empty(max(size, 1), device=DEV)
    lib.vae2_wgrad_defer(1 if deferred else 0)
    try:
        ops.call("vae2_conv2d_bwd_weight_bnin", xp, ctypes.byref(xact), ops.ptr(save_d),
                 relu, dyp, ctypes.byref(dyact), ops.ptr(dw), ops.ptr(db), k, s, pad, acc,
                 ops.ptr(ws), size, ops.stream_ptr())
        if deferred:
            ops.call("vae2_wgrad_flush", ops.stream_ptr())
    finally:
        lib.vae2_wgrad_defer(0)
    torch.cuda.synchronize()
    z = _normalised(_nchw(x), save, relu)
    ref = conv2d_weight(z, (cout, cin, k, k), _nchw(dy), s, pad)
    if acc:
        ref = ref + dw0.cpu()
    assert rel(dw.cpu(), ref) < 1e-4, (key, rel(dw.cpu(), ref))


def _replay_dgrad_bnpart(key, lib):
    """dX of the consumer conv plus the producer BatchNorm's backward partials
    (sum g, sum g*xhat with g = dX masked by the ReLU recomputed from r) from its epilogue:
    dX vs CPU fp32, the partials' sums vs fp64 of the same terms."""
    from vae2 import ops
    _, dya, dyal, dxa, dxal, k, s, pad, bxa, bxal, relu = key
    dy, _ = _buffer(dya, dyal)
    dx, _ = _buffer(dxa, dxal)
    r, _ = _buffer(bxa, bxal)
    cout, cin = dya[3], dxa[3]
    g = torch.Generator().manual_seed(zlib.crc32(repr(key).encode()))
    w = (torch.randn(cout, cin, k, k, generator=g) / (cout * k * k) ** 0.5).to(DEV)
    save = _bn_save(cin, g)
    save_d = save.to(DEV)
    dyp, dyact = ops.act_of(dy)
    dxp, dxact = ops.act_of(dx)
    rp, ract = ops.act_of(r)
    rows = lib.vae2_conv2d_bwd_data_bnpart_rows(dyp, ctypes.byref(dyact), ctypes.byref(dxact), k,
                                                s, pad)
    assert rows > 0, key
    part = torch.empty(2 * rows * cin, device=DEV)
    ops.call("vae2_conv2d_bwd_data_bnpart", dyp, ctypes.byref(dyact),
             ops.ptr(ops.packed_weight(w, 1)), dxp, ctypes.byref(dxact), k, s, pad, rp,
             ctypes.byref(ract), ops.ptr(save_d), relu, ops.ptr(part), ops.stream_ptr())
    torch.cuda.synchronize()
    n, h, wd, _, _ = dxa
    ref = conv2d_input((n, cin, h, wd), w.cpu(), _nchw(dy), s, pad)
    assert rel(_nchw(dx), ref) < 2e-5, (key, rel(_nchw(dx), ref))
    gd = _nchw(dx).double()  # the partials are of the kernel's own dX
    rd = _nchw(r).double()
    sd = save.double()
    if relu:
        gd = torch.where(_normalised(rd, sd, False) > 0, gd, torch.zeros_like(gd))
    xh = (rd - sd[:cin].view(1, cin, 1, 1)) * sd[cin:2 * cin].view(1, cin, 1, 1)
    exact = torch.stack([gd.sum((0, 2, 3)), (gd * xh).sum((0, 2, 3))])
    got = part.view(2, rows, cin).double().sum(1).cpu()
    assert rel(got, exact) < 1e-5, (key, rel(got, exact))


def _kernels(calls, names, fams=None):
    out = set()
    for name, _, ks in calls:
        if name in names:
            out.update(k for k in ks if k and (fams is None or _family(k) in fams))
    return out


def test_conv_instances_at_bench_geometry(bench_step):
    """Every distinct conv call of the bench step replayed at its exact layout against
    torch-CPU fp32, and every conv kernel instance the step launched among those replayed."""
    from vae2 import _lib
    lib = _lib.load()
    keys = []
    for name, desc, _ in bench_step:
        if name in CONV_ABI and desc:
            for kk in desc:
                if kk not in keys:
                    keys.append(kk)
    assert any(k[0] == "fwd" for k in keys) and any(k[0] == "wgrad" for k in keys)
    # the LazyBN calls of the bench step are among the recorded ones (BNX = 1 / 2 kernels)
    assert all(any(k[0] == kind for k in keys)
               for kind in ("fwd_bnin", "wgrad_bnin", "dgrad_bnpart")), sorted({k[0] for k in keys})
    want = _kernels(bench_step, CONV_ABI)
    replay = {"fwd": _replay_fwd, "dgrad": _replay_dgrad, "wgrad": _replay_wgrad,
              "fwd_bnin": _replay_fwd_bnin, "wgrad_bnin": _replay_wgrad_bnin,
              "dgrad_bnpart": _replay_dgrad_bnpart}
    with Recorder() as rec:
        for key in keys:
            replay[key[0]](key, lib)
    got = _kernels(rec.calls, CONV_ABI)
    want = {k for k in want if _family(k) in ("conv_fwd", "conv_dgrad", "conv_wgrad",
                                             "conv_1x1")}
    missing = sorted(want - got)
    assert not missing, missing
    print(f"{len(keys)} distinct conv calls, {len(want)} kernel instances replayed:")
    for k in sorted(want):
        print("  ", k)


def _ref_block_module(m, xs):
    """The reference HighResolutionModule forward (oracle/ref_cpu.py) on NCHW tensors."""
    from oracle import ref_cpu
    return ref_cpu._hr_module(m, xs)


def test_stage4_module_at_bench_geometry(bench_step):
    """A stage-4 HighResolutionModule (4 lock-stepped branches of 2 BasicBlocks, fuse rows
    with 1x1 up paths and stride-2 down chains) at the bench's branch shapes, training
    BatchNorm: outputs, input gradients, weight / BN gradients and running statistics
    against the oracle's reference formulation in fp64 (held to 3x the fp32 formulation's
    own distance, min 1e-4; outputs 1e-4 max-relative)."""
    from vae2 import hrnet
    ed, _ = build(make_cfg(arch="w18", hw=(H, W)))
    mod = ed.stage4[0]
    g = torch.Generator().manual_seed(12)
    with torch.no_grad():  # O(1) activations (the reference init makes BN see ~0)
        for p in mod.modules():
            if isinstance(p, torch.nn.Conv2d):
                p.weight.normal_(0, (1.0 / p.weight[0].numel()) ** 0.5, generator=g)
            elif isinstance(p, torch.nn.BatchNorm2d):
                p.weight.uniform_(0.5, 1.5, generator=g)
                p.bias.normal_(0, 0.1, generator=g)
    shapes = [(18, H, W), (36, H // 2, W // 2), (72, H // 4, W // 4), (144, H // 8, W // 8)]
    xs = [torch.randn(B, c, h, w, generator=g) for c, h, w in shapes]
    m64, m32 = copy.deepcopy(mod).double(), copy.deepcopy(mod)
    x64 = [x.double().requires_grad_() for x in xs]
    x32 = [x.clone().requires_grad_() for x in xs]
    o64 = _ref_block_module(m64, x64)
    o32 = _ref_block_module(m32, x32)
    gouts = [torch.randn(o.shape, generator=g) for o in o64]
    torch.autograd.backward(o64, [go.double() for go in gouts])
    torch.autograd.backward(o32, gouts)
    # the reference's own sensitivity: fp64 runs with 1e-6 relative noise on the inputs
    # (the fp32 forwards here are 2-8e-7 from fp64; every ReLU / fuse mask such an error
    # flips moves the gradients upstream of it by ~1e-3: at 1.2M pre-activations per
    # branch that is a lottery of ~1 flip per run), the largest distance over 4 draws
    sens = []
    for _ in range(4):
        m64p = copy.deepcopy(mod).double()
        x64p = [(x.double() * (1 + 1e-6 * torch.randn(x.shape, generator=g, dtype=torch.float64)))
                .requires_grad_() for x in xs]
        torch.autograd.backward(_ref_block_module(m64p, x64p), [go.double() for go in gouts])
        sens.append((m64p, x64p))
    mg = copy.deepcopy(mod).to(DEV)
    from vae2 import ops
    xg = []
    for x in xs:
        t = ops.new_act((B, x.shape[2], x.shape[3], x.shape[1]), torch.empty(1, device=DEV))
        with torch.no_grad():
            t.copy_(x.permute(0, 2, 3, 1).to(DEV))
        xg.append(t.requires_grad_())
    with Recorder() as rec:
        og = mg.run(xg)
        torch.autograd.backward(og, [go.permute(0, 2, 3, 1).contiguous().to(DEV) for go in gouts])
        torch.cuda.synchronize()
    errs = [max_rel(_nchw(o), r) for o, r in zip(og, o64)]
    assert max(errs) < 1e-4, errs

    rows = [(f"x{i}.grad", rel(_nchw(a.grad), b.grad), rel(c.grad, b.grad),
             max(rel(xp[i].grad, b.grad) for _, xp in sens))
            for i, (a, b, c) in enumerate(zip(xg, x64, x32))]
    sp = [dict(m.named_parameters()) for m, _ in sens]
    rows += [(n, rel(p.grad, p64.grad), rel(p32.grad, p64.grad),
              max(rel(d[n].grad, p64.grad) for d in sp))
             for (n, p), (_, p64), (_, p32) in
             zip(mg.named_parameters(), m64.named_parameters(), m32.named_parameters())]
    for r in rows:
        print(f"{r[0]:40s} hip {r[1]:.3e}  cpu32 {r[2]:.3e}  fp64(x+1e-6) {r[3]:.3e}")
    print("outputs max-rel: hip", [f"{e:.2e}" for e in errs], "cpu32",
          [f"{max_rel(a, b):.2e}" for a, b in zip(o32, o64)])
    # per tensor within 3x the larger of the fp32 formulation's distance and the fp64
    # reference's own sensitivity (min 1e-4); the median within 1.5x of the larger medians
    bad = [r for r in rows if not r[1] < max(1e-4, 3 * max(r[2], r[3]))]
    assert not bad, bad
    import numpy as np
    med = max(np.median([r[2] for r in rows]), np.median([r[3] for r in rows]))
    assert np.median([r[1] for r in rows]) <= 1.5 * med + 1e-6
    for (n, b), (_, b64_) in zip(mg.named_buffers(), m64.named_buffers()):
        if "running" in n:
            assert max_rel(b, b64_) < 1e-5, (n, max_rel(b, b64_))
    # every BatchNorm / fuse kernel instance of the step ran here, except the backward
    # instances specialised for a residual BatchNorm (ResBN, template argument RB = true:
    # the layer-1 Bottleneck's downsample shortcut, not part of a stage-4 module; they run
    # in tests/test_lazy_bn_gpu.py::test_resbn_shortcut_equals_stored)
    import re
    resbn = re.compile(r"bn_bwd_(apply|reduce)_multi_kernel<\d+, true")
    missing = sorted(k for k in _kernels(bench_step, BN_FUSE_ABI) - _kernels(rec.calls, BN_FUSE_ABI)
                     if not resbn.match(k))
    assert not missing, missing


def test_heads_at_bench_geometry(bench_step):
    """The three 270-channel heads (vae2/heads.py: per-branch 1x1 products, up-sum, BN,
    fused output conv, upsampling adjoints) at the bench's branch shapes against the
    reference formulation in fp64 (tests/test_heads_gpu.py's rule), and every head kernel
    instance the step launched among those launched here."""
    from test_heads_gpu import _heads_and_inputs, ref_heads
    from vae2 import heads as vheads
    heads, ys = _heads_and_inputs("w18", (H, W), B, seed=5)
    ref_h = [copy.deepcopy(h).double() for h in heads]
    ys_ref = [y.double().requires_grad_() for y in ys]
    out_ref = ref_heads(ref_h, ys_ref)
    gout = torch.randn(out_ref.shape, generator=torch.Generator().manual_seed(8),
                       dtype=torch.float64)
    (out_ref * gout).sum().backward()
    f32_h = [copy.deepcopy(h).float() for h in heads]
    ys_f32 = [y.clone().requires_grad_() for y in ys]
    (ref_heads(f32_h, ys_f32) * gout.float()).sum().backward()
    hip_h = [copy.deepcopy(h).to(DEV) for h in heads]
    ys_hip = [y.permute(0, 2, 3, 1).contiguous().to(DEV).requires_grad_() for y in ys]
    with Recorder() as rec:
        out = vheads.run(hip_h, ys_hip)
        out.backward(gout.float().permute(0, 2, 3, 1).contiguous().to(DEV))
        torch.cuda.synchronize()
    e = max_rel(_nchw(out), out_ref)
    assert e < 1e-5, e

    rows = [(f"y{i}.grad", rel(_nchw(a.grad), b.grad), rel(c.grad, b.grad))
            for i, (a, b, c) in enumerate(zip(ys_hip, ys_ref, ys_f32))]
    for k, (hh, hr, h32) in enumerate(zip(hip_h, ref_h, f32_h)):
        for (name, p), (_, pr), (_, p32) in zip(hh.named_parameters(), hr.named_parameters(),
                                                h32.named_parameters()):
            if name == "0.bias":  # analytically zero in front of BN
                assert float(p.grad.abs().max()) < 1e-4 * float(hr[0].weight.grad.abs().max())
                continue
            rows.append((f"head{k}.{name}", rel(p.grad, pr.grad), rel(p32.grad, pr.grad)))
    for r in rows:
        print(f"{r[0]:40s} hip {r[1]:.3e}  cpu32 {r[2]:.3e}")
    bad = [r for r in rows if not r[1] < max(1e-4, 3 * r[2])]
    assert not bad, bad
    missing = sorted(_kernels(bench_step, HEAD_ABI) - _kernels(rec.calls, HEAD_ABI))
    assert not missing, missing
