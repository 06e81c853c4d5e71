"""Autograd operators of the VAE² ELBO step, each backed by libvae2_hip kernels.

Activations are NHWC fp32 device tensors of shape (N, H, W, C) whose channel
axis is contiguous (channel slices of a wider buffer are allowed: every kernel
takes the pixel stride).  Parameters keep the reference nn.Conv2d /
nn.BatchNorm2d layouts.

Gradients of parameters that carry a ``main_grad`` attribute (the flat gradient
buffer set up by :mod:`vae2.params`) are accumulated straight into it by the
kernels; parameters without one receive ordinary autograd gradients.

Reference operators replaced (see include/vae2_hip.h for the kernel entry points):
  conv_bn     nn.Conv2d -> nn.BatchNorm2d -> [+residual] -> [nn.ReLU]
              (BasicBlock/Bottleneck enc_hrnet.py:33-103, stems :465-470/:788-793,
              transitions :372-406, fuse branches :177-221, heads :323-370)
  conv        nn.Conv2d with bias, no BN (final head conv, z-net head :1024-1040)
  fuse_sum    HighResolutionModule fuse sum + bilinear upsample + ReLU :233-249
  up_cat      F.upsample(bilinear) of branches 1..3 + torch.cat :833-839
  cat         torch.cat on channels incl. code-map tiling :454-462, :818-830
  avgpool     nn.AdaptiveAvgPool2d((1, 1)) :1025
  l1          L1Loss criterion.py:61-69
  reparam_kl  z = mu + exp(0.5 logvar) eps (utils.py:85-101) + KLLoss criterion.py:72-87
  lsgan       lsgan_adversarial_loss criterion.py:90-103
  split_frames  the discriminator's per-frame slices x[:, 3f:3f+3] (utils.py:116-118)
  weighted_sum  loss assembly utils.py:150-152
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib, prof, streams
from ._lib import Act, call

_F32 = torch.float32


# ----------------------------------------------------------------- helpers ----
def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def act_of(t):
    """(data pointer, Act) of an NHWC activation view."""
    if t.dim() != 4 or t.dtype != _F32 or not t.is_cuda:
        raise ValueError(f"expected a 4-D float32 device tensor (N,H,W,C), got {tuple(t.shape)} "
                         f"{t.dtype} on {t.device}")
    n, h, w, c = t.shape
    s0, s1, s2, s3 = t.stride()
    if c > 1 and s3 != 1:
        raise ValueError("channel axis must be contiguous")
    if w > 1:
        ps = s2
    elif h > 1:
        ps = s1
    elif n > 1:
        ps = s0
    else:
        ps = c
    if (w > 1 and s2 != ps) or (h > 1 and s1 != w * ps) or (n > 1 and s0 != h * w * ps) or ps < c:
        raise ValueError(f"not a uniform NHWC view: shape {tuple(t.shape)} strides {t.stride()}")
    return ctypes.c_void_p(t.data_ptr()), Act(n, h, w, c, ps)


def as_act(t):
    """Return t if it is an NHWC view the kernels accept, else a contiguous copy."""
    try:
        act_of(t)
        return t
    except ValueError:
        return t.contiguous()


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _empty(shape, like, dtype=_F32):
    return torch.empty(shape, dtype=dtype, device=like.device)


def new_act(shape, like):
    """Uninitialised NHWC activation (N,H,W,C) whose pixel stride is rounded up to
    a multiple of 4 channels (16-byte aligned pixels: the conv kernels' vector path)."""
    n, h, w, c = shape
    cp = (c + 3) // 4 * 4
    buf = torch.empty((n, h, w, cp), dtype=_F32, device=like.device)
    return buf if cp == c else buf[..., :c]


def _grad_sink(p, need=True):
    """(buffer to accumulate a parameter gradient into, value autograd should get).
    `need`: ctx.needs_input_grad of the parameter (fixed at forward time, so a
    parameter frozen during the forward — vae2.model.frozen — gets no gradient)."""
    if p is None or not need or not p.requires_grad:
        return None, None
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        return mg, None
    g = torch.zeros_like(p)
    return g, g


def _bn_group():
    from . import dist as vdist
    return vdist.sync_bn_group()


def _all_reduce_sums(sums, count, group):
    if group is None:
        return sums, count
    from . import dist as vdist
    vdist.syncbn_all_reduce_(sums, group=group)  # in place: the callers' sums are fresh buffers
    return sums, count * dist.get_world_size(group)


class GradLink:
    """In-kernel accumulation of the gradient of a tensor with `n` consumers inside one
    block (a residual block's input feeds conv1 and the shortcut).  Each consumer's
    backward writes its contribution into one shared buffer (the first overwrites, the
    others accumulate with beta = 1 in the producing kernel's epilogue) and only the
    last one hands the buffer to autograd (the others return None), so autograd never
    launches an add kernel for it.  Order-agnostic: whichever consumer runs last returns."""

    __slots__ = ("n", "buf", "done")

    def __init__(self, n=2):
        self.n, self.buf, self.done = n, None, 0

    def finish(self):
        self.done += 1
        if self.done < self.n:
            return None
        buf, self.buf = self.buf, None
        return buf


# ------------------------------------------------- BN fused into the consumer ----
class LazyBN:
    """A training-mode BatchNorm(+ReLU) layer whose normalised output z is never stored
    (BasicBlock's bn1 -> relu -> conv2, enc_hrnet.py:46-55): its _ConvBNMulti level
    returns the pre-BN conv output r in z's place, the consumer conv normalises r while
    staging its input (vae2_conv2d_fwd_bnin; the weight gradient likewise,
    vae2_conv2d_bwd_weight_bnin), and the consumer's data gradient -- the gradient of z
    -- writes this layer's backward partials in its epilogue
    (vae2_conv2d_bwd_data_bnpart), so neither the forward apply pass nor the backward
    reduce pass runs for it.  `save` = the layer's (mean, invstd, scale, shift)."""

    __slots__ = ("save", "relu", "part", "rows")

    def __init__(self):
        self.save, self.relu, self.part, self.rows = None, False, None, 0


LAZY_BN = True  # False: every BatchNorm output is stored (A/B and parity tests)


class PartBN:
    """A training-mode BatchNorm(+ReLU) layer without residual whose STORED output y feeds
    exactly one conv that cannot normalise lazily (a 1x1 GEMM, a gather-kernel conv, a
    stride-2 conv): the Bottleneck's bn2 -> conv3 (enc_hrnet.py:84-101), the 144-channel
    branch's BasicBlock bn1 -> conv2, the inner units of a fuse down-chain (:199-218).  The
    forward is unchanged; the consumer's data gradient -- the gradient of y, complete because
    y has no other consumer -- writes this layer's backward partials (sum g, sum g*xhat) in
    its epilogue (vae2_conv2d_bwd_data_bnpart, every kernel family since round 6), so the
    layer's backward reduce pass does not run.  r = the layer's pre-BN tensor (the ReLU mask
    is recomputed from it), save = its (mean, invstd, scale, shift)."""

    __slots__ = ("save", "relu", "part", "rows", "r")

    def __init__(self):
        self.save, self.relu, self.part, self.rows, self.r = None, False, None, 0, None


PART_BN = True  # False: the layers above run their own backward reduce pass (A/B, tests)


class ResBN:
    """Marks a layer of a _ConvBNMulti level whose BatchNorm output (no ReLU) is only the
    residual of another layer of the same level (the Bottleneck's downsample shortcut,
    enc_hrnet.py:94-101): that layer's apply adds it as fma(r, scale, shift) and its
    backward kernels produce this BN's partials and input gradient from the same masked
    gradient (vae2_bn_layer.rx ...), so the shortcut's BN output is never stored and its
    three BN passes do not run."""

    __slots__ = ()


RES_BN = True  # False: the shortcut BN output is stored (A/B and parity tests)
MASK_BYTES = True  # residual layers keep their ReLU mask as bytes for the backward (vs y)
FUSE_LAZY = True   # fuse units' BN outputs formed inside the fuse sum, never stored (A/B)


def lazy_bn_ok(shape, conv):
    """Can `conv` (3x3 stride 1) consume a LazyBN output of NHWC `shape` (N,H,W,C)?
    (the direct 3x3 forward and weight-gradient kernels must run for it)"""
    if not LAZY_BN or not torch.cuda.is_available():
        return False
    n, h, w, c = shape
    k, st, pad = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    if conv.in_channels != c:
        return False
    oh, ow = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    xa = Act(n, h, w, c, (c + 3) // 4 * 4)  # a new_act's layout (16-byte aligned pixels)
    ya = Act(n, oh, ow, conv.out_channels, (conv.out_channels + 3) // 4 * 4)
    return bool(_lib.load().vae2_conv2d_bnin_ok(ctypes.c_void_p(256), ctypes.byref(xa),
                                                ctypes.byref(ya), k, st, pad))


# --------------------------------------------------------------- conv + BN ----
class ConvSpec:
    """Static description of a conv(+BN) call: geometry and module handles."""

    __slots__ = ("k", "stride", "pad", "relu", "bn", "momentum", "eps", "training", "x_link",
                 "res_link", "bn_in", "bn_out", "res_bn", "bn_part")

    def __init__(self, conv, bn=None, relu=False):
        kh, kw = conv.kernel_size
        if kh != kw or conv.stride[0] != conv.stride[1] or conv.padding[0] != conv.padding[1]:
            raise ValueError("only square kernels / strides / paddings are used by the model")
        if conv.groups != 1 or conv.dilation != (1, 1):
            raise ValueError("grouped / dilated convs are not used by the model")
        self.k, self.stride, self.pad = kh, conv.stride[0], conv.padding[0]
        self.relu = relu
        self.bn = bn
        self.x_link = self.res_link = None
        self.bn_in = self.bn_out = None  # LazyBN: BatchNorm fused into the consumer conv
        self.bn_part = None  # PartBN of the producer of x: partials from this conv's dgrad
        self.res_bn = None  # index (in its level) of the layer whose BN output is the residual
        if bn is not None:
            if bn.momentum is None:
                raise ValueError("cumulative-average BatchNorm (momentum=None) is not supported")
            self.momentum = float(bn.momentum)
            self.eps = float(bn.eps)
            self.training = bn.training or not bn.track_running_stats
        else:
            self.momentum = self.eps = 0.0
            self.training = False

    def out_hw(self, h, w):
        return ((h + 2 * self.pad - self.k) // self.stride + 1,
                (w + 2 * self.pad - self.k) // self.stride + 1)


class PackPlan:
    """Every Conv2d weight of a module tree in both packed layouts, refreshed by one
    vae2_conv2d_pack_weights launch (FusedAdam calls run() after each update).

    A conv carrying ``_vae2_col_split`` (a tuple of input-channel block widths: the
    heads, whose 1x1 conv is computed per upsampled branch, vae2.heads) is packed
    per input-channel block instead of whole.

    A weight's packed copy is used only while the weight is unchanged since the
    last run (same storage, same autograd version counter); otherwise the conv
    packs it itself, so in-place edits outside the optimizer stay correct."""

    def __init__(self, module):
        lib = _lib.load()
        seen, self.weights, self.splits = set(), [], []
        for m in module.modules():
            if isinstance(m, torch.nn.Conv2d) and id(m.weight) not in seen:
                seen.add(id(m.weight))
                self.weights.append(m.weight)
                self.splits.append(getattr(m, "_vae2_col_split", None))
        self._blocks, total = [], 0  # per weight: [(c0, cin_block, off0, n0, off1, n1)]
        for w, split in zip(self.weights, self.splits):
            cout, cin, k, _ = w.shape
            blocks, c0 = [], 0
            for cb in (split if split is not None else (cin,)):
                sizes = [lib.vae2_conv2d_packed_size(cout, cb, k, mode) for mode in (0, 1)]
                blocks.append((c0, cb, total, sizes[0], total + sizes[0], sizes[1]))
                total += sizes[0] + sizes[1]
                c0 += cb
            if c0 != cin:
                raise ValueError(f"column split {split} does not cover {cin} input channels")
            self._blocks.append(blocks)
        self.buf = torch.empty((total,), dtype=_F32,
                               device=self.weights[0].device if self.weights else None)
        self._views = [[(self.buf[a:a + na], self.buf[b:b + nb]) for _, _, a, na, b, nb in bl]
                       for bl in self._blocks]
        self._build_jobs()
        self.run()

    def _build_jobs(self):
        if not self.weights:
            self.njobs = 0
            return
        self._ptrs = [w.data_ptr() for w in self.weights]
        jobs = []
        for w, split, blocks, views in zip(self.weights, self.splits, self._blocks, self._views):
            cout, cin, k, _ = w.shape
            ld = cin * k * k if split is not None else 0
            for (c0, cb, *_), vv in zip(blocks, views):
                for mode in (0, 1):
                    jobs.append(_lib.PackJob(w.data_ptr() + 4 * c0 * k * k, vv[mode].data_ptr(),
                                             cout, cb, k, mode, ld, 0))
        arr = (_lib.PackJob * len(jobs))(*jobs)
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.jobs = host.to(self.buf.device)
        self.njobs = len(jobs)

    @torch.no_grad()
    def run(self):
        if not self.weights:
            return
        if any(w.data_ptr() != p for w, p in zip(self.weights, self._ptrs)):
            self._build_jobs()
        call("vae2_conv2d_pack_weights", ptr(self.jobs), self.njobs, stream_ptr())
        for w, split, views in zip(self.weights, self.splits, self._views):
            if split is None:
                w._vae2_packed = (views[0][0], views[0][1], w._version, w.data_ptr())
            else:
                w._vae2_packed_cols = (tuple(split), views, w._version, w.data_ptr())

    def bump_versions(self):
        """Mark the weights modified (an in-place kernel wrote them) and re-pack."""
        torch.autograd.graph.increment_version(self.weights)
        self.run()


def packed_weight(weight, mode):
    """Weights in the kernels' packed layout (mode 0: forward, 1: data gradient)."""
    cached = getattr(weight, "_vae2_packed", None)
    if cached is not None and cached[2] == weight._version and cached[3] == weight.data_ptr():
        return cached[mode]
    cout, cin, k, _ = weight.shape
    out = torch.empty((_lib.load().vae2_conv2d_packed_size(cout, cin, k, mode),),
                      dtype=_F32, device=weight.device)
    call("vae2_conv2d_pack_weight", ptr(weight), cout, cin, k, mode, ptr(out), stream_ptr())
    return out


def packed_weight_cols(weight, split, j, mode):
    """Packed layout of input-channel block j of `weight` under the column split."""
    split = tuple(split)
    cached = getattr(weight, "_vae2_packed_cols", None)
    if (cached is not None and cached[0] == split and cached[2] == weight._version and
            cached[3] == weight.data_ptr()):
        return cached[1][j][mode]
    cout, cin, k, _ = weight.shape
    c0, cb = sum(split[:j]), split[j]
    out = torch.empty((_lib.load().vae2_conv2d_packed_size(cout, cb, k, mode),),
                      dtype=_F32, device=weight.device)
    call("vae2_conv2d_pack_weight_ld", ctypes.c_void_p(weight.data_ptr() + 4 * c0 * k * k),
         cout, cb, k, mode, cin * k * k, ptr(out), stream_ptr())
    return out


def _conv_work(kind, xa, yshape, k, stride):
    """prof.note for a conv call: 2*M*N*K FLOPs; input, output and weights moved once."""
    n, oh, ow, cout = yshape
    prof.note(2.0 * n * oh * ow * cout * xa.c * k * k,
              4.0 * (xa.n * xa.h * xa.w * xa.c + n * oh * ow * cout + cout * xa.c * k * k),
              prof.conv_label(kind, xa.c, cout, k, stride, xa.h, xa.w))


def _conv_fwd(x, weight, bias, spec, stats=None):
    xp, xa = act_of(x)
    n, h, w, _ = x.shape
    oh, ow = spec.out_hw(h, w)
    cout = weight.shape[0]
    y = new_act((n, oh, ow, cout), x)
    yp, ya = act_of(y)
    wp = packed_weight(weight, 0)
    if prof.active():
        _conv_work("fwd", xa, (n, oh, ow, cout), spec.k, spec.stride)
    call("vae2_conv2d_fwd", xp, ctypes.byref(xa), ptr(wp), ptr(bias), yp, ctypes.byref(ya),
         spec.k, spec.stride, spec.pad, 0.0, ptr(stats), stream_ptr())
    return y


class ConvGroup:
    """Independent convolutions of one depth level queued and issued by one
    vae2_conv2d_multi call (direct-3x3 layers share launches).  Tensors a queued job
    uses (packed weights) are held until the call is enqueued; `pending(t)` tells whether
    a queued job writes t's storage (the caller flushes before touching it)."""

    def __init__(self):
        self.jobs, self.hold, self.outs, self.notes = [], [], set(), []

    def add(self, kind, x, xa, wp, bias, y, ya, spec, beta=0.0, stats=None):
        self.jobs.append(_lib.ConvJob(kind, spec.k, spec.stride, spec.pad, x, xa, ptr(wp),
                                      ptr(bias), y, ya, beta, ptr(stats)))
        self.hold.append((wp, bias, stats))
        self.outs.add(y.value if isinstance(y, ctypes.c_void_p) else int(y))
        self.notes.append(prof.take())  # the job's algorithmic work travels with it

    def pending(self, t):
        return t is not None and t.data_ptr() in self.outs

    def flush(self):
        if not self.jobs:
            return
        if prof.active() and not _lib.load().vae2_conv2d_set_grouping(0):
            # profiling, jobs launched one by one anyway (grouping off): one call per job,
            # so each call's time and work are its own kernel's
            for job, work in zip(self.jobs, self.notes):
                prof.put(work)
                call("vae2_conv2d_multi", 1, (_lib.ConvJob * 1)(job), stream_ptr())
        else:
            if prof.active():
                _lib.load().vae2_conv2d_set_grouping(1)
                prof.put(_merge(self.notes))
            arr = (_lib.ConvJob * len(self.jobs))(*self.jobs)
            call("vae2_conv2d_multi", len(self.jobs), arr, stream_ptr())
        self.jobs, self.hold, self.outs, self.notes = [], [], set(), []


def _merge(notes):
    """One note for a grouped launch: work summed, layer shapes joined."""
    notes = [n for n in notes if n is not None]
    if not notes:
        return None
    return (sum(n[0] for n in notes), sum(n[1] for n in notes),
            " + ".join(n[2] for n in notes if n[2]))


def _conv_fwd_queued(group, x, weight, bias, spec, stats, sp=None):
    """_conv_fwd, queued on a ConvGroup (a LazyBN input: launched at once, normalised
    while staged).  group None: launched at once on stream sp (a level lane, see
    _Lanes); the output is allocated on the current stream either way."""
    sp = stream_ptr() if sp is None else sp
    xp, xa = act_of(x)
    n, h, w, _ = x.shape
    oh, ow = spec.out_hw(h, w)
    cout = weight.shape[0]
    y = new_act((n, oh, ow, cout), x)
    yp, ya = act_of(y)
    if prof.active():
        _conv_work("fwd", xa, (n, oh, ow, cout), spec.k, spec.stride)
    lz = spec.bn_in
    if lz is not None:
        call("vae2_conv2d_fwd_bnin", xp, ctypes.byref(xa), ptr(lz.save), int(lz.relu),
             ptr(packed_weight(weight, 0)), ptr(bias), yp, ctypes.byref(ya), spec.k,
             spec.stride, spec.pad, 0.0, ptr(stats), sp)
        return y
    if group is None:
        call("vae2_conv2d_fwd", xp, ctypes.byref(xa), ptr(packed_weight(weight, 0)), ptr(bias),
             yp, ctypes.byref(ya), spec.k, spec.stride, spec.pad, 0.0, ptr(stats), sp)
        return y
    group.add(0, xp, xa, packed_weight(weight, 0), bias, yp, ya, spec, 0.0, stats)
    return y


_WGRAD_BATCH = [0]  # open wgrad_batch contexts
_WS_HOLD = []       # (queueing stream handle, workspace) of queued weight-gradient reductions
_WGRAD_CB = [False, -1]  # end-of-backward flush queued with the engine, by graph task id


def flush_wgrad(own_stream=False):
    """Launch every queued weight-gradient reduction on the current stream, after the
    side streams' work (the convs that wrote the partial slabs), and release the held
    workspaces (recorded on this stream, so the allocator reuses them only after it).
    own_stream: only the reductions queued from the current stream (their slabs were
    written on it: no join), the others stay queued with their workspaces held."""
    cur = torch.cuda.current_stream() if torch.cuda.is_available() else None
    if own_stream:
        key = cur.cuda_stream if cur is not None else None
        # a full flush earlier in this backward may have launched reductions this stream
        # queued on another stream: whatever follows here (vae2.dist.anchor_reduce's
        # all-reduce) is ordered after them
        if _FLUSH_EV[0] is not None and cur is not None:
            cur.wait_event(_FLUSH_EV[0])
        call("vae2_wgrad_flush_stream", stream_ptr())
        keep = [(k, t_) for k, t_ in _WS_HOLD if k != key]
        _WS_HOLD[:] = keep
        return
    streams.join_all()
    try:
        call("vae2_wgrad_flush", stream_ptr())
    finally:
        if cur is not None:
            for _, t_ in _WS_HOLD:
                if t_.is_cuda:
                    t_.record_stream(cur)
            ev = torch.cuda.Event()
            ev.record(cur)
            _FLUSH_EV[0] = ev
        _WS_HOLD.clear()


# completion of the last full flush of the current backward on its launch stream (reset at
# the end of every backward, so a wait never spans steps or a graph capture's boundary)
_FLUSH_EV = [None]


def _end_of_backward():
    _WGRAD_CB[0] = False
    flush_wgrad()
    _FLUSH_EV[0] = None


def _graph_task():
    """Id of the autograd graph task running on this thread (-1 outside a backward)."""
    try:
        return torch._C._current_graph_task_id()
    except (AttributeError, RuntimeError):
        return -1


class wgrad_batch:
    """Context: the weight-gradient slab reductions of the convs in it are queued
    (vae2_wgrad_defer) and launched together, up to 32 per launch, once at the end of
    the backward pass (an autograd engine final callback; the early gradient buckets of
    vae2.dist flush first), or at the context's exit outside a backward.  Their
    workspaces are held until then.  Only reductions into flat-buffer ``main_grad``
    views are deferred: a dW target handed to autograd is reduced at once
    (_defer_off), since autograd reads it as soon as the backward function returns."""

    def __enter__(self):
        if _WGRAD_BATCH[0] == 0 and _WGRAD_CB[0] and _WGRAD_CB[1] != _graph_task():
            # the backward that queued the end-of-backward flush raised before the engine
            # ran its final callbacks (it drops them): flush the stale queue now
            _end_of_backward()
        _lib.load().vae2_wgrad_defer(1)
        _WGRAD_BATCH[0] += 1
        return self

    def __exit__(self, *exc):
        _WGRAD_BATCH[0] -= 1
        if _WGRAD_BATCH[0] == 0:
            _lib.load().vae2_wgrad_defer(0)
            if not _WGRAD_CB[0]:
                try:
                    torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
                    _WGRAD_CB[0], _WGRAD_CB[1] = True, _graph_task()
                except RuntimeError:  # not inside a backward pass: flush now
                    flush_wgrad()
        return False


class _defer_off:
    """The weight-gradient reductions issued inside run now, deferral or not (their dW
    target is not a main_grad view: autograd consumes it when the backward returns)."""

    __slots__ = ("on", "prev")

    def __init__(self, on=True):
        self.on = on

    def __enter__(self):
        if self.on:
            self.prev = _lib.load().vae2_wgrad_defer(0)
        return self

    def __exit__(self, *exc):
        if self.on:
            _lib.load().vae2_wgrad_defer(self.prev)
        return False


def _conv_bwd(x, weight, bias, dy, spec, need_dx, need_w=True, need_b=True, group=None,
              sp=None, hold=None):
    """dW/db accumulated into sinks; returns (dx or None, grad for W, grad for b).  With a
    ConvGroup the data gradient is queued on it (dx is complete once it is flushed).  An
    input marked `_vae2_no_dx` (vae2.dist.anchor_reduce's output when its source needs no
    gradient) gets none: it requires grad only to route the anchor's backward.
    sp: launch on this stream (a level lane, _Lanes) while allocating on the current one;
    the weight-gradient reduction then runs at once on the lane (not deferred: the deferred
    queue is keyed by launch stream) and the workspaces go to `hold`, which the caller keeps
    until the lane has joined."""
    lane = sp is not None
    s = stream_ptr() if sp is None else sp
    xp, xa = act_of(x)
    dyp, dya = act_of(dy)
    wsink, wret = _grad_sink(weight, need_w)
    bsink, bret = _grad_sink(bias, need_b)
    if wsink is not None or bsink is not None:
        tmp_w = wsink is None
        if tmp_w:  # weight frozen but bias trained: still need a dW target
            wsink = torch.zeros_like(weight)
        size = _lib.load().vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xa), ctypes.byref(dya),
                                                          spec.k)
        ws = _empty((max(size, 1),), x)
        if prof.active():
            _conv_work("wgrad", xa, tuple(dy.shape), spec.k, spec.stride)
        lz = spec.bn_in
        now = wret is not None or tmp_w or lane  # not a main_grad view: reduce before returning
        if lane and hold is not None:
            hold.append(ws)
        with _defer_off(now and _WGRAD_BATCH[0] > 0):
            if lz is not None:
                call("vae2_conv2d_bwd_weight_bnin", xp, ctypes.byref(xa), ptr(lz.save),
                     int(lz.relu), dyp, ctypes.byref(dya), ptr(wsink), ptr(bsink), spec.k,
                     spec.stride, spec.pad, 1, ptr(ws), size, s)
            else:
                call("vae2_conv2d_bwd_weight", xp, ctypes.byref(xa), dyp, ctypes.byref(dya),
                     ptr(wsink), ptr(bsink), spec.k, spec.stride, spec.pad, 1, ptr(ws), size, s)
        if _WGRAD_BATCH[0] and not now:  # the deferred reduction reads it at the flush
            _WS_HOLD.append((torch.cuda.current_stream().cuda_stream, ws))
    dx = None
    if need_dx and not getattr(x, "_vae2_no_dx", False):
        link = spec.x_link
        beta = 0.0
        if link is not None and link.buf is not None:
            dx, beta = link.buf, 1.0  # accumulate onto the other consumer's contribution
        else:
            dx = new_act(tuple(x.shape), x)
            if link is not None:
                link.buf = dx
        dxp, dxa = act_of(dx)
        wp = packed_weight(weight, 1)
        if prof.active():
            _conv_work("dgrad", xa, tuple(dy.shape), spec.k, spec.stride)
        lz = spec.bn_in
        pb = spec.bn_part
        if pb is not None and (pb.r is None or pb.save is None or link is not None):
            pb = None  # the producer stored no pre-BN tensor, or x has another consumer
        rows = 0
        if (lz is not None or pb is not None) and beta == 0.0:
            rows = _lib.load().vae2_conv2d_bwd_data_bnpart_rows(
                dyp, ctypes.byref(dya), ctypes.byref(dxa), spec.k, spec.stride, spec.pad)
        if rows > 0:  # + the producer layer's backward partials (its reduce pass skipped)
            part = _empty((2 * rows * xa.c,), x)
            if hold is not None:
                hold.append(part)
            src = lz if lz is not None else pb
            # the producer's pre-BN tensor: x itself for a LazyBN input, r for a PartBN one
            bxp, bxa = (xp, xa) if lz is not None else act_of(pb.r)
            call("vae2_conv2d_bwd_data_bnpart", dyp, ctypes.byref(dya), ptr(wp), dxp,
                 ctypes.byref(dxa), spec.k, spec.stride, spec.pad, bxp, ctypes.byref(bxa),
                 ptr(src.save), int(src.relu), ptr(part), s)
            src.part, src.rows = part, rows
        elif group is not None:
            group.add(1, dyp, dya, wp, None, dxp, dxa, spec, beta)
        else:
            call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dya), ptr(wp), dxp,
                 ctypes.byref(dxa), spec.k, spec.stride, spec.pad, beta, s)
        if link is not None:
            dx = link.finish()
    return dx, wret, bret


class _ConvBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, residual, spec):
        lib = _lib.load()
        s = stream_ptr()
        bn = spec.bn
        n, h, w, _ = x.shape
        oh, ow = spec.out_hw(h, w)
        cout = weight.shape[0]
        count = float(n * oh * ow)
        group = None
        if spec.training:
            xp, xa = act_of(x)
            rows = lib.vae2_conv2d_fwd_stats_rows(xp, ctypes.byref(xa),
                                                  ctypes.byref(Act(n, oh, ow, cout, cout)),
                                                  spec.k, spec.stride, spec.pad)
            stats = _empty((2 * rows * cout,), x)
            r = _conv_fwd(x, weight, bias, spec, stats)
            sums = _empty((2 * cout,), x, torch.float64)
            group = _bn_group()
            save = _empty((4 * cout,), x)
            track = bn.track_running_stats and bn.running_mean is not None
            stat_ptrs = (ptr(bn.running_mean) if track else None,
                         ptr(bn.running_var) if track else None,
                         ptr(bn.num_batches_tracked) if track else None)
            if group is None:
                if count <= 1:
                    raise ValueError("Expected more than 1 value per channel when training, "
                                     f"got input size {(n, cout, oh, ow)}")
                call("vae2_bn_reduce_finalize", ptr(stats), rows, cout, ptr(sums), count,
                     ptr(gamma), ptr(beta), *stat_ptrs, spec.momentum, spec.eps, ptr(save), s)
            else:  # SyncBN: exchange the double sums between the reduction and finalize
                call("vae2_bn_partials_reduce", ptr(stats), rows, cout, ptr(sums), 0, s)
                sums, count = _all_reduce_sums(sums, count, group)
                if count <= 1:
                    raise ValueError("Expected more than 1 value per channel when training")
                call("vae2_bn_finalize", ptr(sums), count, ptr(gamma), ptr(beta), *stat_ptrs,
                     spec.momentum, spec.eps, cout, ptr(save), s)
        else:
            r = _conv_fwd(x, weight, bias, spec)
            save = _empty((4 * cout,), x)
            call("vae2_bn_eval_coeffs", ptr(gamma), ptr(beta), ptr(bn.running_mean),
                 ptr(bn.running_var), spec.eps, cout, ptr(save), s)
        y = new_act((n, oh, ow, cout), x)
        rp, ra = act_of(r)
        yp, ya = act_of(y)
        if residual is not None:
            resp, resa = act_of(residual)
        else:
            resp, resa = None, ya
        if prof.active():  # read r (+ residual), write y
            prof.note(0, 4.0 * r.numel() * (3 if residual is not None else 2))
        call("vae2_bn_apply", rp, ctypes.byref(ra), ptr(save), resp, ctypes.byref(resa), yp,
             ctypes.byref(ya), int(spec.relu), s)
        ctx.spec = spec
        ctx.count = count
        ctx.group = group
        ctx.has_res = residual is not None
        ctx.params = (weight, bias, gamma, beta)
        ctx.save_for_backward(x, r, y, save)
        return y

    @staticmethod
    def backward(ctx, dy):
        if not ctx.spec.training:
            raise RuntimeError("backward through an eval-mode BatchNorm is not supported")
        lib = _lib.load()
        s = stream_ptr()
        x, r, y, save = ctx.saved_tensors
        weight, bias, gamma, beta = ctx.params
        spec = ctx.spec
        dy = as_act(dy)
        cout = r.shape[3]
        dyp, dya = act_of(dy)
        rp, ra = act_of(r)
        yp, ya = act_of(y)
        if not ctx.has_res:
            yp = None  # the kernels recompute the ReLU mask from r (no read of y)
        rows = lib.vae2_bn_partial_rows(ctypes.byref(ra))
        part = _empty((2 * rows * cout,), r)
        if prof.active():  # read dy, r (+ y)
            prof.note(0, 4.0 * r.numel() * (3 if yp is not None else 2))
        call("vae2_bn_relu_bwd_reduce", dyp, ctypes.byref(dya), yp, ctypes.byref(ya), rp,
             ctypes.byref(ra), ptr(save), int(spec.relu), ptr(part), s)
        lsums = _empty((2 * cout,), r, torch.float64)
        gsink, gret = _grad_sink(gamma, ctx.needs_input_grad[3])
        bsink, bret = _grad_sink(beta, ctx.needs_input_grad[4])
        call("vae2_bn_bwd_reduce_param_grads", ptr(part), rows, cout, ptr(lsums), ptr(gsink),
             ptr(bsink), s)
        gsums, _ = _all_reduce_sums(lsums, ctx.count, ctx.group)
        dr = new_act(tuple(r.shape), r)
        drp, dra = act_of(dr)
        dres = None
        link = spec.res_link
        if ctx.has_res and ctx.needs_input_grad[5]:
            dres = new_act(tuple(r.shape), r)
            dresp, dresa = act_of(dres)
        else:
            dresp, dresa = None, dra
        if prof.active():  # read dy, r (+ y); write dr (+ dres)
            prof.note(0, 4.0 * r.numel() * (3 + (1 if yp is not None else 0) +
                                             (1 if dres is not None else 0)))
        call("vae2_bn_relu_bwd_apply", dyp, ctypes.byref(dya), yp, ctypes.byref(ya), rp,
             ctypes.byref(ra), ptr(save), ptr(gamma), ptr(gsums), ctx.count, int(spec.relu), drp,
             ctypes.byref(dra), dresp, ctypes.byref(dresa), s)
        if dres is not None and link is not None:
            if link.buf is None:
                link.buf = dres
            else:  # (not reached by the blocks: conv1's backward runs after this one)
                link.buf.add_(dres)
            dres = link.finish()
        dx, wret, bret_conv = _conv_bwd(x, weight, bias, dr, spec, ctx.needs_input_grad[0],
                                        ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return dx, wret, bret_conv, gret, bret, dres, None


def conv_bn(x, conv, bn, relu, residual=None, x_link=None, res_link=None, bn_part=None):
    """relu?(bn(conv(x)) + residual) with training-mode (or eval-mode) BatchNorm.
    x_link / res_link: GradLink shared with the other consumer(s) of x / residual.
    bn_part: the PartBN of the layer that produced x (its partials from this conv's data
    gradient).  Training mode goes through the multi-layer path (one layer); eval mode, and
    residual views the multi-layer kernels cannot take, through _ConvBN."""
    spec = ConvSpec(conv, bn, relu)
    spec.x_link, spec.res_link = x_link, res_link
    spec.bn_part = bn_part if PART_BN else None
    if spec.training and (residual is None or _bn_quad_ok(residual)):
        return _ConvBNMulti.apply((spec,), x, conv.weight, conv.bias, bn.weight, bn.bias,
                                  residual)[0]
    return _ConvBN.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, residual, spec)


def _bn_quad_ok(t):
    """Eligible for the multi-layer BN kernels: 16-byte aligned, pixel stride % 4 == 0."""
    p_, a = act_of(t)
    return p_.value % 16 == 0 and a.ps % 4 == 0 and a.c <= 1024


_COUNTS = {}


def _counts_dev(counts, like):
    """Device copy of per-layer element counts (cached: the SyncBN exchange appends
    them to the statistics so the global count is the sum of the real local counts)."""
    key = (tuple(counts), like.device)
    t = _COUNTS.get(key)
    if t is None:
        t = torch.tensor(counts, dtype=torch.float64).to(like.device)
        _COUNTS[key] = t
    return t


LEVEL_LANES = 0  # concurrent lanes per depth level inside a graph capture (0/1: off; measured slower)
LEVEL_LANES_BWD = True  # lanes in the backward as well


class _Lanes:
    """The independent convolutions of one depth level on concurrent streams while a HIP
    graph is captured (the lock-stepped HRNet branches: 18@128x256, 36@64x128, 72@32x64,
    144@16x32 -- the same FLOPs each, but the 72 / 144-channel layers fill a quarter of the
    chip on their own).  In the replayed graph the level is a fork/join of independent
    kernel nodes, so the narrow layers run side by side.  Lane 0 is the current (parent)
    stream; lane k > 0 a stream of its own per (parent, k), forked from the parent before
    the level and joined into it after.  Every buffer is allocated on the parent stream and
    kept alive until the join (callers hold them), so the allocator never sees lane uses.
    Layers whose data gradients accumulate into one buffer (a shared GradLink) share a lane.
    Eager steps and profiled steps keep one stream (a stream switch costs host time there)."""

    def __init__(self, specs, enabled=True):
        self.on = False
        self.lane = [0] * len(specs)
        if (not enabled or LEVEL_LANES <= 1 or len(specs) < 2 or not torch.cuda.is_available()
                or prof.active()):
            return
        keys = []
        for i, sp in enumerate(specs):
            key = id(sp.x_link) if sp.x_link is not None else ("solo", i)
            if key not in keys:
                keys.append(key)
            self.lane[i] = keys.index(key) % LEVEL_LANES
        if max(self.lane) == 0:
            return
        self.parent = torch.cuda.current_stream()
        # only the main (capture) stream forks lanes: a second-level fork -- lanes forked
        # from a side stream that is itself forked from the capture stream (the posterior
        # net's, the past decoder's) -- makes HIP's stream-capture end segfault (ROCm 7.0
        # runtime; reproduced with plain torch ops by scripts/probe_lane_capture.py, nest
        # mode); those sub-networks already run beside the main stream's work
        if streams.role_of(self.parent) != "main":
            return
        # the lane streams exist before the capture (created by the eager warm-up steps)
        self.streams = {k: streams.side_stream(self.parent.device, ("lane", "main", k))
                        for k in sorted(set(self.lane) - {0})}
        self.on = torch.cuda.is_current_stream_capturing()
        if not self.on:
            return
        for st in self.streams.values():
            st.wait_stream(self.parent)
            streams._FORKED.add(st)

    def ptr(self, i):
        """Launch stream of layer i (None: the current stream)."""
        if not self.on or self.lane[i] == 0:
            return None
        return ctypes.c_void_p(self.streams[self.lane[i]].cuda_stream)

    def join(self):
        if self.on:
            for st in self.streams.values():
                self.parent.wait_stream(st)

    def sync(self):
        """Join, then fork again: parent work issued now is ordered with every lane's work
        before and after it."""
        if self.on:
            self.join()
            for st in self.streams.values():
                st.wait_stream(self.parent)


class _ConvBNMulti(torch.autograd.Function):
    """n independent conv -> BatchNorm(train) [-> +residual] [-> ReLU] layers (one HRNet
    depth level): the convs launch per layer, every BatchNorm step is one launch for all
    n layers (vae2_bn_multi_*), and with SyncBN one exchange carries all n layers'
    statistics and element counts.  flat = (x, weight, bias, gamma, beta, residual) per
    layer."""

    @staticmethod
    def forward(ctx, specs, *flat):
        lib = _lib.load()
        s = stream_ptr()
        n = len(specs)
        L = [flat[6 * i:6 * i + 6] for i in range(n)]
        group = _bn_group()
        rs, saves, fins, counts, cs = [], [], [], [], []
        lanes = _Lanes(specs)
        cg = None if lanes.on else ConvGroup()
        for li, ((x, weight, bias, gamma, beta, residual), spec) in enumerate(zip(L, specs)):
            nn_, h, w, _ = x.shape
            oh, ow = spec.out_hw(h, w)
            cout = weight.shape[0]
            xp, xa = act_of(x)
            rows = lib.vae2_conv2d_fwd_stats_rows(xp, ctypes.byref(xa),
                                                  ctypes.byref(Act(nn_, oh, ow, cout, cout)),
                                                  spec.k, spec.stride, spec.pad)
            stats = _empty((2 * rows * cout,), x)
            rs.append(_conv_fwd_queued(cg, x, weight, bias, spec, stats, lanes.ptr(li)))
            saves.append(_empty((4 * cout,), x))
            counts.append(float(nn_ * oh * ow))
            cs.append(cout)
            fins.append((stats, rows))
        if cg is not None:
            cg.flush()  # the level's convs: direct-3x3 layers share launches
        lanes.join()
        tot = 2 * sum(cs)
        buf = _empty((tot + n,), rs[0], torch.float64)
        world = 1
        if group is not None:
            buf[tot:].copy_(_counts_dev(counts, buf))
            world = dist.get_world_size(group)
        arr = (_lib.BnFin * n)()
        off = 0
        for i, ((stats, rows), spec, c) in enumerate(zip(fins, specs, cs)):
            bn = spec.bn
            gamma, beta = L[i][3], L[i][4]
            if counts[i] * world <= 1:
                raise ValueError("Expected more than 1 value per channel when training, "
                                 f"got input size {(counts[i], c)}")
            track = bn.track_running_stats and bn.running_mean is not None
            arr[i] = _lib.BnFin(
                stats.data_ptr(), rows, c, buf.data_ptr() + 8 * off,
                buf.data_ptr() + 8 * (tot + i) if group is not None else None, counts[i],
                _p(gamma), _p(beta), _p(bn.running_mean) if track else None,
                _p(bn.running_var) if track else None,
                _p(bn.num_batches_tracked) if track else None, spec.momentum, spec.eps,
                saves[i].data_ptr(), None, None)
            off += 2 * c
        if group is None:
            call("vae2_bn_multi_reduce", n, arr, 0, s)
        else:  # SyncBN: one exchange of every layer's (sum x, sum x^2) and count
            call("vae2_bn_multi_reduce", n, arr, 2, s)
            from . import dist as vdist
            vdist.syncbn_all_reduce_(buf, group=group)
            call("vae2_bn_multi_finalize", n, arr, s)
        ys, lay = [], []
        masks = [None] * n
        for i, (r, save, spec) in enumerate(zip(rs, saves, specs)):
            lz = spec.bn_out
            if isinstance(lz, ResBN):  # added by its consumer's apply: r stands in for y
                ys.append(r)
                continue
            if isinstance(lz, PartBN):  # y stored as usual; the consumer's data gradient
                ok = L[i][5] is None and spec.res_bn is None  # will write the partials
                lz.save, lz.relu, lz.part, lz.rows = save, spec.relu, None, 0
                lz.r = r if ok else None
                lz = None
            if lz is not None:  # normalised by the consumer conv: r stands in for y
                lz.save, lz.relu, lz.part, lz.rows = save, spec.relu, None, 0
                ys.append(r)
                continue
            y = new_act(tuple(r.shape), r)
            ys.append(y)
            res = L[i][5]
            layer = _bn_layer(r, res, y, None, None, save, None, None, None, None, 0.0,
                              spec.relu)
            if MASK_BYTES and spec.relu and (res is not None or spec.res_bn is not None):
                # the backward's ReLU mask (it cannot be recomputed from r): 1 byte per
                # channel quad instead of re-reading y twice
                _, ya_ = act_of(y)
                mk = torch.empty((ya_.n * ya_.h * ya_.w * ((ya_.c + 3) // 4),),
                                 dtype=torch.uint8, device=y.device)
                layer.mask = mk.data_ptr()
                masks[i] = mk
            if spec.res_bn is not None:
                j = spec.res_bn
                layer.rx, layer.rxd = rs[j].data_ptr(), act_of(rs[j])[1]
                layer.rsave = saves[j].data_ptr()
            lay.append(layer)
        if lay:
            if prof.active():
                prof.note(0, sum(4.0 * r.numel() * (3 if L[i][5] is not None or
                                                    specs[i].res_bn is not None else 2)
                                 for i, r in enumerate(rs) if specs[i].bn_out is None),
                          _bn_label("bn apply", [rs[i] for i in range(n)
                                                 if specs[i].bn_out is None]))
            call("vae2_bn_multi_apply", len(lay), (_lib.BnLayer * len(lay))(*lay), s)
        ctx.specs = specs
        ctx.masks = masks
        ctx.counts = counts
        ctx.group = group
        ctx.has_res = [l_[5] is not None for l_ in L]
        ctx.params = [l_[1:5] for l_ in L]
        ctx.save_for_backward(*[l_[0] for l_ in L], *rs, *ys, *saves)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        s = stream_ptr()
        specs = ctx.specs
        n = len(specs)
        saved = ctx.saved_tensors
        xs, rs, ys, saves = (saved[k * n:(k + 1) * n] for k in range(4))
        need = ctx.needs_input_grad
        cs = [int(r.shape[3]) for r in rs]
        tot = 2 * sum(cs)
        buf = _empty((tot + n,), rs[0], torch.float64)
        group = ctx.group
        if group is not None:
            buf[tot:].copy_(_counts_dev(ctx.counts, buf))
        lay = (_lib.BnLayer * n)()
        fins = (_lib.BnFin * n)()
        keep, drs, dress, red = [], [], [], []
        off = 0
        lib = _lib.load()
        # a shortcut BN (ResBN) gets its partials / input gradient from its consumer's
        # kernels: its buffers first, so the consumer's layer can point at them
        resbuf, o_ = {}, 0
        for i in range(n):
            if isinstance(specs[i].bn_out, ResBN):
                _, ra = act_of(rs[i])
                rows = lib.vae2_bn_partial_rows(ctypes.byref(ra))
                resbuf[i] = (_empty((2 * rows * cs[i],), rs[i]), rows,
                             new_act(tuple(rs[i].shape), rs[i]), buf.data_ptr() + 8 * o_)
            o_ += 2 * cs[i]
        act = []  # layers with BN passes of their own (not ResBN)
        for i in range(n):
            r, y, save, spec = rs[i], ys[i], saves[i], specs[i]
            if i in resbuf:
                part, rows, dr, sums_p = resbuf[i]
                gamma, beta = ctx.params[i][2], ctx.params[i][3]
                gsink, gret = _grad_sink(gamma, need[1 + 6 * i + 3])
                bsink, bret = _grad_sink(beta, need[1 + 6 * i + 4])
                fins[i] = _lib.BnFin(part.data_ptr(), rows, cs[i], sums_p, None, ctx.counts[i],
                                     None, None, None, None, None, 0.0, 0.0, None, _p(gsink),
                                     _p(bsink))
                keep.append((part,))
                drs.append(dr)
                dress.append((None, gret, bret))
                off += 2 * cs[i]
                continue
            act.append(i)
            dy = dys[i]
            dy = as_act(dy) if dy is not None else torch.zeros_like(y)
            if not _bn_quad_ok(dy):  # e.g. a channel slice of a concatenation's gradient
                dy = _aligned_copy(dy)
            lz = spec.bn_out
            pre = lz is not None and lz.part is not None and dys[i] is not None
            if pre:  # partials from the consumer's data-gradient epilogue
                part, rows = lz.part, lz.rows
                lz.part = None
            else:
                _, ra = act_of(r)
                rows = lib.vae2_bn_partial_rows(ctypes.byref(ra))
                part = _empty((2 * rows * cs[i],), r)
                red.append(i)
            dr = new_act(tuple(r.shape), r)
            dres, acc = None, 0
            if ctx.has_res[i] and need[1 + 6 * i + 5]:
                link = spec.res_link
                if (link is not None and link.buf is not None and
                        tuple(link.buf.shape) == tuple(r.shape) and _bn_quad_ok(link.buf)):
                    dres, acc = link.buf, 1  # summed onto the other consumer's gradient in-kernel
                else:
                    dres = new_act(tuple(r.shape), r)
            gamma, beta = ctx.params[i][2], ctx.params[i][3]
            gsink, gret = _grad_sink(gamma, need[1 + 6 * i + 3])
            bsink, bret = _grad_sink(beta, need[1 + 6 * i + 4])
            sums_p = buf.data_ptr() + 8 * off
            countp = buf.data_ptr() + 8 * (tot + i) if group is not None else None
            mk = ctx.masks[i]
            lay[i] = _bn_layer(r, y if (ctx.has_res[i] or spec.res_bn is not None) and mk is None
                               else None, dr, dy, dres, save, gamma, part, sums_p, countp,
                               ctx.counts[i], spec.relu, acc)
            if mk is not None:
                lay[i].mask = mk.data_ptr()
            if spec.res_bn is not None:  # the shortcut BN's passes ride on this layer's
                j = spec.res_bn
                rpart, _, rdr, rsums_p = resbuf[j]
                lay[i].rx, lay[i].rxd = rs[j].data_ptr(), act_of(rs[j])[1]
                lay[i].rsave = saves[j].data_ptr()
                lay[i].rgamma = _p(ctx.params[j][2])
                lay[i].rpartials, lay[i].rsums = rpart.data_ptr(), rsums_p
                lay[i].rdx, lay[i].rdxd = rdr.data_ptr(), act_of(rdr)[1]
            fins[i] = _lib.BnFin(part.data_ptr(), rows, cs[i], sums_p, None, ctx.counts[i],
                                 None, None, None, None, None, 0.0, 0.0, None, _p(gsink),
                                 _p(bsink))
            keep.append((dy, part))
            drs.append(dr)
            dress.append((dres, gret, bret))
            off += 2 * cs[i]
        if red:
            if prof.active():
                prof.note(0, sum(4.0 * rs[i].numel() * (2 + _y_reads(ctx, i) +
                                                        (1 if specs[i].res_bn is not None else 0))
                                 for i in red), _bn_label("bn bwd reduce", [rs[i] for i in red]))
            call("vae2_bn_multi_bwd_reduce", len(red), (_lib.BnLayer * len(red))(*[lay[i] for i in red]),
                 s)
        call("vae2_bn_multi_reduce", n, fins, 1, s)  # local sums + dgamma / dbeta
        if group is not None:  # SyncBN: global (sum g, sum g*xhat) for the input gradients
            from . import dist as vdist
            vdist.syncbn_all_reduce_(buf, group=group)
        if prof.active():
            prof.note(0, sum(4.0 * rs[i].numel() * (3 + _y_reads(ctx, i) +
                                                    (1 if dress[i][0] is not None else 0) +
                                                    (2 if specs[i].res_bn is not None else 0))
                             for i in act), _bn_label("bn bwd apply", [rs[i] for i in act]))
        call("vae2_bn_multi_bwd_apply", len(act), (_lib.BnLayer * len(act))(*[lay[i] for i in act]),
             s)
        grads = [None]
        lanes = _Lanes(specs, LEVEL_LANES_BWD)
        # the level's data gradients: direct-3x3 layers share launches (one stream), or the
        # layers run on concurrent lanes (graph capture)
        cg = None if lanes.on else ConvGroup()
        hold = []
        with wgrad_batch():  # the level's weight-gradient reductions in one launch
            for i in range(n):
                spec = specs[i]
                x = xs[i]
                weight, bias = ctx.params[i][0], ctx.params[i][1]
                dres, gret, bret = dress[i]
                link = spec.res_link
                if dres is not None and link is not None:
                    if link.buf is None:
                        link.buf = dres
                    elif link.buf is not dres:  # (dres is link.buf: summed in the BN kernel)
                        if cg is not None and cg.pending(link.buf):
                            cg.flush()
                        if lanes.on:  # a lane may still be writing it
                            lanes.sync()
                        link.buf.add_(dres)
                    dres = link.finish()
                dx, wret, bret_conv = _conv_bwd(x, weight, bias, drs[i], spec, need[1 + 6 * i],
                                                need[1 + 6 * i + 1], need[1 + 6 * i + 2],
                                                group=cg, sp=lanes.ptr(i), hold=hold)
                grads += [dx, wret, bret_conv, gret, bret, dres]
            if cg is not None:
                cg.flush()
            lanes.join()
        del hold  # (after the join: the lanes' workspaces return to the parent's pool)
        return tuple(grads)


def _p(t):
    return t.data_ptr() if t is not None else None


def _y_reads(ctx, i):
    """Bytes (in units of the layer's fp32 tensor) a backward pass reads for the ReLU mask:
    y, its byte mask (1/16), or nothing (recomputed from r)."""
    if ctx.masks[i] is not None:
        return 1.0 / 16.0
    return 1 if ctx.has_res[i] or ctx.specs[i].res_bn is not None else 0


def _bn_label(kind, rs):
    """Profiler row label of a multi-layer BN launch: its layers' C@HxW (N in the bytes)."""
    return f"{kind} " + " + ".join(f"{int(r.shape[3])}@{int(r.shape[1])}x{int(r.shape[2])}"
                                   for r in rs)


def _aligned_copy(t):
    out = new_act(tuple(t.shape), t)
    tp, ta = act_of(t)
    op, oa = act_of(out)
    call("vae2_copy_act", tp, ctypes.byref(ta), op, ctypes.byref(oa), 0.0, stream_ptr())
    return out


def _bn_layer(x, a, o, dy, dres, save, gamma, part, sums_p, countp, count, relu, dres_acc=0):
    def d(t):
        return act_of(t)[1] if t is not None else Act(0, 0, 0, 0, 0)
    return _lib.BnLayer(_p(x), d(x), _p(a), d(a), _p(o), d(o), _p(dy), d(dy), _p(dres), d(dres),
                        _p(save), _p(gamma), _p(part), sums_p, countp, float(count), int(relu),
                        int(dres_acc))


BN_BATCH = True  # False: conv_bn_multi runs its layers one by one (A/B and parity tests)


def conv_bn_multi(xs, convs, bns, relu, residuals=None, x_links=None, res_links=None,
                  bn_outs=None, bn_ins=None, res_bns=None):
    """[conv_bn(xs[i], convs[i], bns[i], relu, residuals[i], ...)] for independent layers,
    their BatchNorm steps batched into shared launches (training mode; with SyncBN one
    statistics exchange per direction for all of them).

    bn_outs[i] (a LazyBN, or None): layer i's BatchNorm output is consumed only by a conv
    that takes it lazily -- the returned tensor is then the pre-BN conv output, to be
    passed on with bn_ins[i] = that LazyBN to the consumer's conv_bn_multi call.  Where
    the batched path does not run, the entry is set to None (the output is stored).
    A PartBN entry instead keeps the stored output and, passed on as the consumer's
    bn_ins[i], makes the consumer's data gradient write layer i's backward partials.

    res_bns[i] (an index j, or None): layer i's residual is layer j's BatchNorm output
    (layer j: no ReLU, no residual of its own, same output shape), added in layer i's
    apply and never stored (ResBN); layer j's entry of the returned list is then its
    pre-BN conv output, for no other use."""
    n = len(xs)
    residuals = residuals if residuals is not None else [None] * n
    x_links = x_links if x_links is not None else [None] * n
    res_links = res_links if res_links is not None else [None] * n
    relus = relu if isinstance(relu, (list, tuple)) else [relu] * n
    specs = []
    for i in range(n):
        spec = ConvSpec(convs[i], bns[i], relus[i])
        spec.x_link, spec.res_link = x_links[i], res_links[i]
        if bn_outs is not None:
            spec.bn_out = bn_outs[i]
        if bn_ins is not None:
            if isinstance(bn_ins[i], PartBN):  # stored input, partials from the dgrad
                spec.bn_part = bn_ins[i] if PART_BN else None
            else:
                spec.bn_in = bn_ins[i]
        specs.append(spec)
    if res_bns is not None:
        for i, j in enumerate(res_bns):
            if j is None:
                continue
            if (residuals[i] is not None or residuals[j] is not None or relus[j] or
                    res_bns[j] is not None or (bn_outs is not None and
                                               (bn_outs[i] is not None or bn_outs[j] is not None))):
                raise ValueError("res_bns: the shortcut layer must be a plain conv + BN")
            shp = [(xs[k].shape[0], *specs[k].out_hw(xs[k].shape[1], xs[k].shape[2]),
                    convs[k].out_channels) for k in (i, j)]
            if shp[0] != shp[1]:
                raise ValueError(f"res_bns: shortcut output {shp[1]} != layer output {shp[0]}")
            specs[i].res_bn = j
            specs[j].bn_out = ResBN()
    if (not BN_BATCH or not RES_BN and res_bns is not None and any(j is not None for j in res_bns)
            or not all(sp.training for sp in specs) or
            not all(r is None or _bn_quad_ok(r) for r in residuals)):
        if any(sp.bn_in is not None for sp in specs):
            raise RuntimeError("a LazyBN input needs the batched training path")
        if bn_outs is not None:
            bn_outs[:] = [None] * n
        outs = [None] * n
        order = [j for j in range(n) if res_bns is not None and j in res_bns]
        order += [i for i in range(n) if i not in order]
        for i in order:  # shortcut layers first: stored, then used as the residual
            res = residuals[i]
            if res_bns is not None and res_bns[i] is not None:
                res = outs[res_bns[i]]
            outs[i] = conv_bn(xs[i], convs[i], bns[i], relus[i], res, x_links[i], res_links[i])
        return outs
    flat = []
    for i in range(n):
        flat += [xs[i], convs[i].weight, convs[i].bias, bns[i].weight, bns[i].bias, residuals[i]]
    return list(_ConvBNMulti.apply(tuple(specs), *flat))


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, spec):
        y = _conv_fwd(x, weight, bias, spec)
        ctx.spec = spec
        ctx.params = (weight, bias)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        weight, bias = ctx.params
        dx, wret, bret = _conv_bwd(x, weight, bias, as_act(dy), ctx.spec, ctx.needs_input_grad[0],
                                   ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return dx, wret, bret, None


def conv(x, conv_mod):
    """nn.Conv2d forward (with its bias), no normalisation."""
    return _Conv.apply(x, conv_mod.weight, conv_mod.bias, ConvSpec(conv_mod))


# ------------------------------------------------------------- fuse / cat ----
def _up_bwd(g, shape):
    dx = new_act(shape, g)
    gp, ga = act_of(g)
    dxp, dxa = act_of(dx)
    call("vae2_upsample_bilinear_bwd", gp, ctypes.byref(ga), dxp, ctypes.byref(dxa), 0.0,
         stream_ptr())
    return dx


UP_POW2 = True  # the fuse rows' lower-branch adjoints in two launches (exact 2/4/8 ratios)


def _up_bwd_pow2(g, shapes):
    """Adjoints of up to 3 upsample terms at once (vae2_upsample_bilinear_bwd_pow2), or
    None when the ratios are not exact powers of two (callers take _up_bwd per term)."""
    if not UP_POW2 or len(shapes) > 3:
        return None
    lib = _lib.load()
    gp, ga = act_of(g)
    dxs = [new_act(shp, g) for shp in shapes]
    views = [act_of(d) for d in dxs]
    acts = (Act * len(dxs))(*[a for _, a in views])
    wsz = lib.vae2_upsample_bilinear_bwd_pow2_ws_size(ctypes.byref(ga), len(dxs), acts)
    if wsz < 0 or ga.ps % 4 or g.data_ptr() % 16:
        return None
    ptrs = (ctypes.c_void_p * len(dxs))(*[p for p, _ in views])
    ws = _empty((max(wsz, 1),), g)
    call("vae2_upsample_bilinear_bwd_pow2", gp, ctypes.byref(ga), len(dxs), ptrs, acts, None,
         ptr(ws), wsz, stream_ptr())
    return dxs


class _FuseSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out_hw, links, lazies, *terms):
        ref = terms[0]
        n, c = ref.shape[0], ref.shape[3]
        y = new_act((n, out_hw[0], out_hw[1], c), ref)
        ptrs = (ctypes.c_void_p * len(terms))()
        acts = (Act * len(terms))()
        for i, t in enumerate(terms):
            p_, a_ = act_of(t)
            ptrs[i] = p_
            acts[i] = a_
        yp, ya = act_of(y)
        if lazies is not None and any(lz is not None for lz in lazies):
            # terms that are a fuse unit's pre-BN output, normalised here (never stored)
            sv = (ctypes.c_void_p * len(terms))(*[ptr(lz.save) if lz is not None else None
                                                  for lz in lazies])
            call("vae2_fuse_sum_relu_bn", len(terms), ptrs, acts, sv, yp, ctypes.byref(ya),
                 stream_ptr())
        else:
            call("vae2_fuse_sum_relu", len(terms), ptrs, acts, yp, ctypes.byref(ya),
                 stream_ptr())
        ctx.shapes = [tuple(t.shape) for t in terms]
        ctx.links = links
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = as_act(dy)
        g = new_act(tuple(y.shape), y)
        dyp, dya = act_of(dy)
        yp, ya = act_of(y)
        gp, ga = act_of(g)
        links = ctx.links or (None,) * len(ctx.shapes)
        lk = next((i for i, l in enumerate(links) if l is not None), None)
        if lk is not None and ctx.needs_input_grad[lk + 3]:
            # the identity term's input has other consumers (ops.GradLink): its share of
            # the gradient goes straight into (or onto) their shared buffer
            link = links[lk]
            beta = 0.0
            if link.buf is None:
                link.buf = new_act(tuple(y.shape), y)
            else:
                beta = 1.0
            bp, ba = act_of(link.buf)
            call("vae2_relu_bwd_dual", dyp, ctypes.byref(dya), yp, ctypes.byref(ya), gp,
                 ctypes.byref(ga), bp, ctypes.byref(ba), beta, stream_ptr())
        else:
            lk = None
            call("vae2_relu_bwd", dyp, ctypes.byref(dya), yp, ctypes.byref(ya), gp,
                 ctypes.byref(ga), stream_ptr())
        grads = []
        ups = [i for i, shp in enumerate(ctx.shapes)
               if ctx.needs_input_grad[i + 3] and i != lk and shp[1:3] != tuple(y.shape[1:3])]
        upg = _up_bwd_pow2(g, [ctx.shapes[i] for i in ups]) if ups else None
        for i, shp in enumerate(ctx.shapes):
            if not ctx.needs_input_grad[i + 3]:
                grads.append(None)
            elif i == lk:
                grads.append(links[i].finish())
            elif shp[1:3] == tuple(y.shape[1:3]):
                grads.append(g)
            elif upg is not None:
                grads.append(upg[ups.index(i)])
            else:
                grads.append(_up_bwd(g, shp))
        return (None, None, None, *grads)


def fuse_sum_relu(terms, out_hw, links=None, lazies=None):
    """relu(sum of terms), lower-resolution terms bilinearly upsampled to out_hw.  links:
    per term an ops.GradLink (or None) shared with the term's other consumers.  lazies:
    per term a LazyBN (or None): the term is that BatchNorm layer's pre-BN output, its
    normalised output (the fuse unit's BN, no ReLU) is formed here and never stored; the
    gradient returned for the term is the one of that normalised output (LazyBN's rule)."""
    return _FuseSum.apply(tuple(out_hw), tuple(links) if links else None,
                          tuple(lazies) if lazies else None, *terms)


class _UpCat(torch.autograd.Function):
    """cat([x0, up(x1), up(x2), ...], channels) at x0's resolution."""

    @staticmethod
    def forward(ctx, *xs):
        x0 = xs[0]
        n, h, w, _ = x0.shape
        ctot = sum(t.shape[3] for t in xs)
        y = new_act((n, h, w, ctot), x0)
        s = stream_ptr()
        off = 0
        for t in xs:
            c = t.shape[3]
            dst = y[..., off:off + c]
            tp, ta = act_of(t)
            dp_, da = act_of(dst)
            if t.shape[1:3] == x0.shape[1:3]:
                call("vae2_copy_act", tp, ctypes.byref(ta), dp_, ctypes.byref(da), 0.0, s)
            else:
                call("vae2_upsample_bilinear_fwd", tp, ctypes.byref(ta), dp_, ctypes.byref(da), 0.0,
                     s)
            off += c
        ctx.shapes = [tuple(t.shape) for t in xs]
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = as_act(dy)
        grads = []
        off = 0
        for i, shp in enumerate(ctx.shapes):
            c = shp[3]
            sl = dy[..., off:off + c]
            off += c
            if not ctx.needs_input_grad[i]:
                grads.append(None)
            elif shp[1:3] == tuple(dy.shape[1:3]):
                grads.append(sl)
            else:
                grads.append(_up_bwd(sl, shp))
        return tuple(grads)


def up_cat(xs):
    return _UpCat.apply(*xs)


class _Cat(torch.autograd.Function):
    """Channel concat of NHWC maps and per-clip vectors tiled over space.

    parts: tensors that are either NHWC maps (N,h,w,c) at the output resolution or
    per-clip vectors given as (N,1,1,c) maps with tile=True.
    """

    @staticmethod
    def forward(ctx, out_hw, tiles, *parts):
        ref = parts[0]
        n = ref.shape[0]
        ctot = sum(p_.shape[3] for p_ in parts)
        y = new_act((n, out_hw[0], out_hw[1], ctot), ref)
        s = stream_ptr()
        off = 0
        for p_, tile in zip(parts, tiles):
            c = p_.shape[3]
            dst = y[..., off:off + c]
            dp_, da = act_of(dst)
            pp, pa = act_of(p_)
            if tile:
                call("vae2_codemap_tile_fwd", pp, pa.ps, dp_, ctypes.byref(da), s)
            else:
                call("vae2_copy_act", pp, ctypes.byref(pa), dp_, ctypes.byref(da), 0.0, s)
            off += c
        ctx.tiles = tiles
        ctx.shapes = [tuple(p_.shape) for p_ in parts]
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = as_act(dy)
        grads = []
        off = 0
        lib = _lib.load()
        for i, (shp, tile) in enumerate(zip(ctx.shapes, ctx.tiles)):
            c = shp[3]
            sl = dy[..., off:off + c]
            off += c
            if not ctx.needs_input_grad[i + 2]:
                grads.append(None)
            elif tile:
                g = _empty(shp, dy)
                sp, sa = act_of(sl)
                wsz = lib.vae2_spatial_ws_size(ctypes.byref(sa))
                ws = _empty((max(wsz, 1),), dy)
                gp, ga = act_of(g)
                call("vae2_codemap_tile_bwd", sp, ctypes.byref(sa), gp, ga.ps, 0, ptr(ws), wsz,
                     stream_ptr())
                grads.append(g)
            else:
                grads.append(sl)
        return (None, None, *grads)


def cat(parts, out_hw, tiles=None):
    tiles = tuple(tiles) if tiles is not None else (False,) * len(parts)
    return _Cat.apply(tuple(out_hw), tiles, *parts)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n, h, w, c = x.shape
        y = _empty((n, 1, 1, c), x)
        xp, xa = act_of(x)
        yp, ya = act_of(y)
        wsz = _lib.load().vae2_spatial_ws_size(ctypes.byref(xa))
        ws = _empty((max(wsz, 1),), x)
        call("vae2_global_avgpool_fwd", xp, ctypes.byref(xa), yp, ctypes.byref(ya), ptr(ws), wsz,
             stream_ptr())
        ctx.shape = tuple(x.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = as_act(dy)
        dx = new_act(ctx.shape, dy)
        dyp, dya = act_of(dy)
        dxp, dxa = act_of(dx)
        call("vae2_global_avgpool_bwd", dyp, ctypes.byref(dya), dxp, ctypes.byref(dxa), 0.0,
             stream_ptr())
        return dx


def avgpool(x):
    return _AvgPool.apply(x)


_POOLW = {}


def _pool_weights(n_in, n_out, device):
    """Sum over the n_out outputs of each input's bilinear weight (align_corners=False,
    F.upsample's index rule in fp32: src = max(0, (o + 0.5) * n_in / n_out - 0.5))."""
    key = (n_in, n_out, str(device))
    t = _POOLW.get(key)
    if t is None:
        import numpy as np
        w = np.zeros(n_in, dtype=np.float64)
        scale = np.float32(n_in) / np.float32(n_out)
        for o in range(n_out):
            src = max(np.float32(0.0), np.float32(scale * np.float32(o + 0.5) - np.float32(0.5)))
            i0 = int(src)
            l1 = float(src - np.float32(i0))
            i1 = i0 + 1 if i0 < n_in - 1 else i0
            w[i0] += 1.0 - l1
            w[i1] += l1
        t = torch.tensor(w, dtype=torch.float32, device=device)
        _POOLW[key] = t
    return t


class _UpAvgPool(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) of cat([x0, up(x1), up(x2), ...]) at x0's resolution
    (enc_hrnet.py:1022-1025): the upsampled branches are pooled at their own resolution
    with the bilinear weights' column sums, so the full-resolution concatenation (and its
    gradient) is never materialised."""

    @staticmethod
    def forward(ctx, *xs):
        x0 = xs[0]
        n, H, W, _ = x0.shape
        ctot = sum(t.shape[3] for t in xs)
        y = _empty((n, 1, 1, ctot), x0)
        s = stream_ptr()
        scale = 1.0 / (H * W)
        off = 0
        ws_keep = []
        for t in xs:
            c = t.shape[3]
            tp, ta = act_of(t)
            ya = Act(n, 1, 1, c, ctot)
            yp = ctypes.c_void_p(y.data_ptr() + 4 * off)
            wsz = _lib.load().vae2_spatial_ws_size(ctypes.byref(ta))
            ws = _empty((max(wsz, 1),), x0)
            ws_keep.append(ws)
            if t.shape[1:3] == x0.shape[1:3]:
                call("vae2_global_avgpool_fwd", tp, ctypes.byref(ta), yp, ctypes.byref(ya),
                     ptr(ws), wsz, s)
            else:
                wr = _pool_weights(t.shape[1], H, x0.device)
                wc = _pool_weights(t.shape[2], W, x0.device)
                call("vae2_weighted_avgpool_fwd", tp, ctypes.byref(ta), ptr(wr), ptr(wc),
                     scale, yp, ctypes.byref(ya), ptr(ws), wsz, s)
            off += c
        ctx.shapes = [tuple(t.shape) for t in xs]
        ctx.hw = (H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        H, W = ctx.hw
        s = stream_ptr()
        ctot = dy.shape[3]
        grads = []
        off = 0
        for i, shp in enumerate(ctx.shapes):
            c = shp[3]
            if not ctx.needs_input_grad[i]:
                grads.append(None)
                off += c
                continue
            dx = new_act(shp, dy)
            dxp, dxa = act_of(dx)
            da = Act(shp[0], 1, 1, c, ctot)
            dp_ = ctypes.c_void_p(dy.data_ptr() + 4 * off)
            if shp[1:3] == (H, W):
                call("vae2_global_avgpool_bwd", dp_, ctypes.byref(da), dxp, ctypes.byref(dxa),
                     0.0, s)
            else:
                wr = _pool_weights(shp[1], H, dy.device)
                wc = _pool_weights(shp[2], W, dy.device)
                call("vae2_weighted_avgpool_bwd", dp_, ctypes.byref(da), ptr(wr), ptr(wc),
                     1.0 / (H * W), dxp, ctypes.byref(dxa), 0.0, s)
            grads.append(dx)
            off += c
        return tuple(grads)


UP_AVGPOOL = True  # False: materialise up_cat(xs) then avgpool (A/B and parity tests)


def up_avgpool(xs):
    """avgpool(up_cat(xs)) without the full-resolution concatenation."""
    if not UP_AVGPOOL:
        return avgpool(up_cat(xs))
    return _UpAvgPool.apply(*xs)


# ---------------------------------------------------------------- layout ----
class _ToNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        n, c, h, w = x.shape
        y = new_act((n, h, w, c), x)
        yp, ya = act_of(y)
        call("vae2_nchw_to_nhwc", ptr(x), yp, ctypes.byref(ya), 0.0, stream_ptr())
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = as_act(dy)
        n, h, w, c = dy.shape
        dx = _empty((n, c, h, w), dy)
        dyp, dya = act_of(dy)
        call("vae2_nhwc_to_nchw", dyp, ctypes.byref(dya), ptr(dx), 0.0, stream_ptr())
        return dx


class _ToNCHW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n, h, w, c = x.shape
        y = _empty((n, c, h, w), x)
        xp, xa = act_of(x)
        call("vae2_nhwc_to_nchw", xp, ctypes.byref(xa), ptr(y), 0.0, stream_ptr())
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        n, c, h, w = dy.shape
        dx = new_act((n, h, w, c), dy)
        dxp, dxa = act_of(dx)
        call("vae2_nchw_to_nhwc", ptr(dy), dxp, ctypes.byref(dxa), 0.0, stream_ptr())
        return dx


def to_nhwc(x):
    return _ToNHWC.apply(x)


def to_nchw(x):
    return _ToNCHW.apply(x)


# ------------------------------------------------------------------ ELBO ----
def _flat_act(t):
    """Describe a dense tensor of any layout as an (1,1,numel,1) activation (for
    element-wise-and-sum kernels whose result does not depend on layout)."""
    t = t.contiguous()
    return t, Act(1, 1, t.numel(), 1, 1)


class _L1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, t, scale, flat):
        if flat:
            p, pa = _flat_act(p)
            t, ta = _flat_act(t)
            pp, tp = ptr(p), ptr(t)
        else:
            pp, pa = act_of(p)
            tp, ta = act_of(t)
        n = pa.n * pa.h * pa.w * pa.c
        ws = _empty((_lib.load().vae2_reduce_ws_size(n),), p)
        out = _empty((), p)
        call("vae2_l1_fwd", pp, ctypes.byref(pa), tp, ctypes.byref(ta), scale, ptr(ws), ptr(out),
             stream_ptr())
        ctx.scale = scale
        ctx.flat = flat
        ctx.save_for_backward(p, t)
        return out

    @staticmethod
    def backward(ctx, gout):
        p, t = ctx.saved_tensors
        gout = gout.contiguous()
        if ctx.flat:
            _, pa = _flat_act(p)
            _, ta = _flat_act(t)
            dp = torch.empty_like(p)
            _, da = _flat_act(dp)
            pp, tp, dpp = ptr(p), ptr(t), ptr(dp)
        else:
            pp, pa = act_of(p)
            tp, ta = act_of(t)
            dp = new_act(tuple(p.shape), p)
            dpp, da = act_of(dp)
        call("vae2_l1_bwd", pp, ctypes.byref(pa), tp, ctypes.byref(ta), ptr(gout), ctx.scale, dpp,
             ctypes.byref(da), 0.0, stream_ptr())
        return dp, None, None, None


def l1(pred, target, scale, flat=False):
    """scale * sum |pred - target| (NHWC views, or any dense layout with flat=True)."""
    return _L1.apply(pred, target, float(scale), flat)


class _LSGAN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target, scale, flat):
        if flat:
            x, xa = _flat_act(x)
            xp = ptr(x)
        else:
            xp, xa = act_of(x)
        ws = _empty((_lib.load().vae2_reduce_ws_size(xa.n * xa.h * xa.w * xa.c),), x)
        out = _empty((), x)
        call("vae2_lsgan_fwd", xp, ctypes.byref(xa), target, scale, ptr(ws), ptr(out),
             stream_ptr())
        ctx.target, ctx.scale, ctx.flat = target, scale, flat
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, gout):
        (x,) = ctx.saved_tensors
        gout = gout.contiguous()
        if ctx.flat:
            _, xa = _flat_act(x)
            dx = torch.empty_like(x)
            xp, dxp, dxa = ptr(x), ptr(dx), xa
        else:
            xp, xa = act_of(x)
            dx = new_act(tuple(x.shape), x)
            dxp, dxa = act_of(dx)
        call("vae2_lsgan_bwd", xp, ctypes.byref(xa), ctx.target, ptr(gout), ctx.scale, dxp,
             ctypes.byref(dxa), 0.0, stream_ptr())
        return dx, None, None, None


def lsgan(sample, real, scale, flat=False):
    """scale * sum (sample - (1 if real else 0))^2  (LSGAN, criterion.py:90-103)."""
    return _LSGAN.apply(sample, 1.0 if real else 0.0, float(scale), flat)


class _SplitFrames(torch.autograd.Function):
    """x (N,H,W,C) -> nframes contiguous (N,H,W,3) maps x[..., 3f:3f+3]; the backward
    writes every frame gradient into one dx (no autograd slice/add kernels)."""

    @staticmethod
    def forward(ctx, x, nframes):
        n, h, w, c = x.shape
        if 3 * nframes > c:
            raise ValueError(f"{nframes} RGB frames do not fit {c} channels (the reference's "
                             "frame loop needs CLIP_LENGTH 3 or more, utils.py:116)")
        s = stream_ptr()
        outs = []
        for f in range(nframes):
            o = new_act((n, h, w, 3), x)
            sp, sa = act_of(x[..., 3 * f:3 * f + 3])
            op, oa = act_of(o)
            call("vae2_copy_act", sp, ctypes.byref(sa), op, ctypes.byref(oa), 0.0, s)
            outs.append(o)
        ctx.shape = tuple(x.shape)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        n, h, w, c = ctx.shape
        ref = next(g for g in gs if g is not None)
        dx = new_act(ctx.shape, ref)
        if 3 * len(gs) < c or any(g is None for g in gs):
            dx.zero_()
        s = stream_ptr()
        for f, g in enumerate(gs):
            if g is None:
                continue
            g = as_act(g)
            gp, ga = act_of(g)
            dp_, da = act_of(dx[..., 3 * f:3 * f + 3])
            call("vae2_copy_act", gp, ctypes.byref(ga), dp_, ctypes.byref(da), 0.0, s)
        return dx, None


def split_frames(x, nframes):
    return _SplitFrames.apply(x, int(nframes))


class _ReparamKL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, muvar, eps, prior, scale):
        n, h, w, c2 = muvar.shape
        zc = c2 // 2
        z = new_act((n, h, w, zc), muvar)
        kl = _empty((), muvar)
        mp, ma = act_of(muvar)
        ep, ea = act_of(eps)
        zp, za = act_of(z)
        ws = _empty((_lib.load().vae2_reduce_ws_size(n * h * w * zc),), muvar)
        call("vae2_reparam_kl_fwd", mp, ctypes.byref(ma), ep, ctypes.byref(ea), zp, ctypes.byref(za),
             int(prior), scale, ptr(kl), 0, ptr(ws), stream_ptr())
        ctx.scale = scale
        ctx.prior = prior
        ctx.save_for_backward(muvar, eps)
        return z, kl

    @staticmethod
    def backward(ctx, dz, dkl):
        muvar, eps = ctx.saved_tensors
        dm = new_act(tuple(muvar.shape), muvar)
        mp, ma = act_of(muvar)
        ep, ea = act_of(eps)
        dmp, dma = act_of(dm)
        if dz is not None and not ctx.prior:
            dz = as_act(dz)
            dzp, dza = act_of(dz)
        else:
            dzp, dza = None, ea
        gk = dkl.contiguous() if dkl is not None else None
        call("vae2_reparam_kl_bwd", mp, ctypes.byref(ma), ep, ctypes.byref(ea), dzp, ctypes.byref(dza),
             ptr(gk), ctx.scale, dmp, ctypes.byref(dma), stream_ptr())
        return dm, None, None, None


def reparam_kl(muvar, eps, prior=False, scale=1.0):
    """(z, KL): z = mu + exp(0.5 logvar) eps (or eps when prior), KL*scale."""
    return _ReparamKL.apply(muvar, eps, bool(prior), float(scale))


class _WeightedSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lambdas, *terms):
        n = len(terms)
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in terms])
        lams = (ctypes.c_float * n)(*lambdas)
        out = _empty((), terms[0])
        call("vae2_weighted_sum", n, ptrs, lams, ptr(out), stream_ptr())
        ctx.lambdas = lambdas
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        grads = []
        for i, lam in enumerate(ctx.lambdas):
            if not ctx.needs_input_grad[i + 1]:
                grads.append(None)
                continue
            d = torch.empty_like(g)
            call("vae2_scale", ptr(d), ptr(g), 1, float(lam), stream_ptr())
            grads.append(d)
        return (None, *grads)


def weighted_sum(terms, lambdas):
    return _WeightedSum.apply(tuple(float(x) for x in lambdas), *terms)


def nonfinite_flag(tensors, flag=None):
    """Device flag (int32) set when any tensor holds a NaN/Inf (no host sync)."""
    if flag is None:
        flag = torch.zeros((1,), dtype=torch.int32, device=tensors[0].device)
    for t in tensors:
        t = t.detach()
        if not t.is_contiguous():
            t = t.contiguous()
        call("vae2_nonfinite_check", ptr(t), t.numel(), ptr(flag), stream_ptr())
    return flag
