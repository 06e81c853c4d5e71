"""Data-parallel runtime: RCCL gradient all-reduce and SyncBatchNorm statistics.

Replaces DistributedDataParallel + nn.SyncBatchNorm.convert_sync_batchnorm
(tools/train.py:107-111, :216-229) and reduce_tensor (function.py:32-43).
One process per GPU; the "nccl" backend of PyTorch-ROCm is RCCL over xGMI.

* SyncBN: every BatchNorm forward all-reduces its per-channel (sum x, sum x^2)
  doubles, every backward its (sum g, sum g*xhat) doubles, so statistics are
  global exactly as with SyncBatchNorm; parameter gradients use local sums and
  are averaged by the gradient all-reduce, as DDP does.
* Gradients: the flat gradient buffer of each model is all-reduced (sum) in
  buckets and scaled by 1/world in a HIP kernel (DDP's mean).  The decoders' range
  of the encoder-decoder buffer (its tail: decf_* / decp_* parameters) is final as
  soon as the gradient of the encoder output x2t_hat is (every decoder node feeds
  it), so a hook on that tensor starts its buckets then, on a communicator of their
  own, while the encoder and posterior backward still run (DDP's bucket overlap
  without per-parameter hooks: the HIP kernels accumulate into the flat buffer).
  SyncBN exchanges stay on the default communicator, so they never queue behind a
  gradient bucket.
"""
import os

import torch
import torch.distributed as dist

from . import ops, streams
from ._lib import call

_SYNC_BN_GROUP = None
_SYNC_BN = False
_GRAD_GROUP = None
_EARLY = {}       # id(flat) -> (flat, end offset already launched, [async works])
FORCE = False     # the distributed code path at world size 1 (tests: bit-identity)
OVERLAP = True    # early decoder buckets (A/B: off = everything after backward)
EARLY_CHECK = None  # tests: a list the early hook appends (flat grad, start, tail snapshot) to


def is_dist():
    return (dist.is_available() and dist.is_initialized() and
            (dist.get_world_size() > 1 or FORCE))


def world_size():
    return dist.get_world_size() if is_dist() else 1


def rank():
    return dist.get_rank() if is_dist() else 0


def init(backend=None):
    """Initialise the process group from torchrun's env (MASTER_ADDR/PORT, RANK, WORLD_SIZE)."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or dist.is_initialized():
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        prepare_nccl_env()
    dist.init_process_group(backend=backend, init_method="env://")


def set_sync_bn(enabled, group=None):
    """Enable global batch statistics (the reference's SyncBatchNorm conversion)."""
    global _SYNC_BN, _SYNC_BN_GROUP
    _SYNC_BN = bool(enabled)
    _SYNC_BN_GROUP = group


def sync_bn_group():
    if not _SYNC_BN or not is_dist():
        return None
    return _SYNC_BN_GROUP if _SYNC_BN_GROUP is not None else dist.group.WORLD


BUCKET_ELEMS = 8 * 1024 * 1024  # 32 MB fp32 buckets


def all_reduce_(t, group=None):
    """In-place sum all-reduce.  RCCL ("nccl") reduces device buffers directly; a gloo
    group (CPU CI, several ranks sharing one GPU) is fed through host staging."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)


# ---- SyncBN statistics: one-shot IPC peer all-reduce (vae2_syncbn_allreduce) ----
SB_MAX_ELEMS = 1 << 15  # doubles per exchange (a depth level's sums: <= 6 x 2 x 512 + 6)


class IpcExchange:
    """The one-shot peer all-reduce of one SyncBN group (csrc/syncbn.hip).  Every exchange
    runs on one dedicated stream in host issue order (the same order on every rank): the
    kernel's sequence numbers pair each exchange with the peers' same exchange even when
    the step issues them from several streams (posterior net, past decoder)."""

    def __init__(self, comm, group, max_elems):
        self.comm, self.group, self.max_elems = comm, group, max_elems
        self.stream = torch.cuda.Stream()

    def takes(self, t, group=None):
        return (t.is_cuda and t.dtype == torch.float64 and t.numel() <= self.max_elems and
                t.is_contiguous() and (group is None or group is self.group or group == self.group))

    def all_reduce_(self, t):
        import ctypes
        cur, cs = torch.cuda.current_stream(), self.stream
        cs.wait_stream(cur)
        call("vae2_syncbn_allreduce", self.comm, ctypes.c_void_p(t.data_ptr()), t.numel(),
             ctypes.c_void_p(cs.cuda_stream))
        cur.wait_stream(cs)

    def error(self):
        """Nonzero once an exchange timed out (sticky: every later exchange of this comm
        writes NaN and exchanges nothing).  Synchronous read of the device error word."""
        import ctypes
        err = ctypes.c_int64(0)
        call("vae2_syncbn_comm_error", self.comm, ctypes.byref(err))
        return err.value

    def set_timeout(self, seconds):
        call("vae2_syncbn_comm_set_timeout", self.comm, float(seconds))


_SB = None  # the active IpcExchange (or a test double with the same methods)


def init_syncbn_ipc(group=None, max_elems=SB_MAX_ELEMS):
    """Route the SyncBN statistics exchanges of `group` (default: the SyncBN group) through
    the one-shot peer all-reduce kernel (csrc/syncbn.hip) instead of RCCL: one kernel per
    exchange, every rank's payload stored into every rank's IPC-mapped receive area over
    xGMI, summed in rank order.  Collective over the group; node-local ranks only
    (LOCAL_WORLD_SIZE == world).  A self-check exchange of rank-dependent values must give
    the exact sums on every rank, else RCCL stays in use.  Returns True when active."""
    global _SB
    import ctypes
    from ._lib import load
    if not is_dist():
        return False
    g = group if group is not None else (sync_bn_group() or dist.group.WORLD)
    if dist.get_backend(g) == "gloo" and not FORCE_IPC:
        return False
    world, rk = dist.get_world_size(g), dist.get_rank(g)
    if world > 8 or int(os.environ.get("LOCAL_WORLD_SIZE", world)) != dist.get_world_size():
        return False  # (several nodes: IPC maps only the node's own GPUs)
    lib = load()
    comm = ctypes.c_void_p()
    h = ctypes.create_string_buffer(64)
    ok = lib.vae2_syncbn_comm_init(rk, world, max_elems, h, ctypes.byref(comm)) == 0
    hs = [None] * world
    dist.all_gather_object(hs, h.raw if ok else None, group=g)
    if all(x is not None for x in hs):
        ok = ok and lib.vae2_syncbn_comm_connect(comm, b"".join(hs)) == 0
    else:
        ok = False
    if ok:  # self-check: exact small-integer sums, every rank
        t = torch.arange(1, 65, dtype=torch.float64, device=torch.cuda.current_device()) * (rk + 1)
        ok = lib.vae2_syncbn_allreduce(comm, ctypes.c_void_p(t.data_ptr()), t.numel(),
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
        torch.cuda.synchronize()
        err = ctypes.c_int64(0)
        lib.vae2_syncbn_comm_error(comm, ctypes.byref(err))
        want = torch.arange(1, 65, dtype=torch.float64) * (world * (world + 1) / 2)
        ok = ok and err.value == 0 and torch.equal(t.cpu(), want)
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok), group=g)
    if not all(flags):
        if comm.value:
            lib.vae2_syncbn_comm_destroy(comm)
        return False
    _SB = IpcExchange(comm, g, max_elems)
    return True


FORCE_IPC = False  # tests: the IPC exchange under a gloo group (ranks sharing one GPU)


def prepare_nccl_env():
    """Environment for a NCCL (RCCL) process group whose steps are captured as HIP graphs:
    ProcessGroupNCCL's CUDA-event cache off (an event of an eager collective must never be
    re-recorded inside a capture while the watchdog may still query it) and its flight
    recorder on (vae2.graph drains the watchdog before a capture by reading which eager
    collectives it has retired).  Call before torch.distributed.init_process_group; an
    explicit setting wins."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    if "TORCH_NCCL_TRACE_BUFFER_SIZE" not in os.environ:
        os.environ.setdefault("TORCH_FR_BUFFER_SIZE", "2000")


def syncbn_exchange():
    """'ipc' when the one-shot peer all-reduce carries the SyncBN statistics, else 'rccl' /
    the group's backend."""
    return "ipc" if _SB is not None else (dist.get_backend(sync_bn_group())
                                          if sync_bn_group() is not None else "none")


def syncbn_all_reduce_(t, group=None):
    """In-place sum of a SyncBN statistics buffer over the SyncBN group (float64)."""
    if _SB is not None and _SB.takes(t, group):
        _SB.all_reduce_(t)
        return
    all_reduce_(t, group=group)


class SyncBNExchangeError(RuntimeError):
    pass


def syncbn_check():
    """Raise SyncBNExchangeError if a SyncBN exchange timed out (a peer did not arrive within
    the kernel's bound; the kernel gave up instead of hanging, wrote NaN statistics and stays
    failed).  Synchronous; the training loop calls it at every PRINT_FREQ point and at the
    end of each epoch (vae2/trainer.py), bench.py after its timed region."""
    if _SB is None:
        return
    if _SB.error():
        raise SyncBNExchangeError(
            "SyncBN IPC exchange timed out (a rank did not arrive): the batch statistics "
            "since then are NaN on this rank and every later exchange fails; restart from "
            "the last checkpoint")


def bucket_allreduce(buf, bucket_elems=BUCKET_ELEMS, group=None):
    """Sum-all-reduce a flat buffer in fixed-size buckets (same bucket boundaries on
    every rank, issued in order)."""
    n = buf.numel()
    for off in range(0, n, bucket_elems):
        all_reduce_(buf[off:off + bucket_elems], group=group)


def grad_group():
    """The gradient buckets' communicator (created once, collectively, on first use)."""
    global _GRAD_GROUP
    if _GRAD_GROUP is None:
        _GRAD_GROUP = dist.new_group(backend=dist.get_backend())
    return _GRAD_GROUP


def tail_range(flat, prefixes=("decf_", "decp_")):
    """First offset of the trailing parameters whose names start with `prefixes`
    (None unless every parameter from there on does)."""
    idx = [i for i, n in enumerate(flat.names) if n.startswith(prefixes)]
    if not idx or idx != list(range(idx[0], len(flat.names))):
        return None
    return flat.offsets[idx[0]]


def _start_range(flat, lo, hi, own_stream=False):
    """Flush the queued weight-gradient reductions, join the side streams, then start the
    bucketed all-reduce of flat.grad[lo:hi] (recorded in _EARLY for allreduce_grads).
    own_stream: the range is written only by work issued on the current stream (a
    sub-network on its own side stream): flush that stream's reductions, no join -- a
    join would not order this stream after a HIP graph's capture stream, whose queued
    reductions a full flush would launch here."""
    if own_stream:
        ops.flush_wgrad(own_stream=True)
    else:
        ops.flush_wgrad()   # queued weight-gradient reductions (they write the range)
        streams.join_all()  # side-stream work (the posterior net, the past decoder)
    buf = flat.grad
    if EARLY_CHECK is not None:  # the range as the buckets see it (no later write allowed)
        EARLY_CHECK.append((buf, lo, hi, buf[lo:hi].clone()))
    works = [dist.all_reduce(buf[off:min(off + BUCKET_ELEMS, hi)], group=grad_group(),
                             async_op=True)
             for off in range(lo, hi, BUCKET_ELEMS)]
    _EARLY.setdefault(id(flat), []).append((lo, hi, works))


def _overlap_ok():
    return OVERLAP and is_dist() and dist.get_backend(grad_group()) != "gloo"


def early_reduce_hook(t, flat, start):
    """Start the all-reduce of flat.grad[start:] when t's gradient is complete."""
    if not (_overlap_ok() and t.requires_grad and start is not None):
        return  # (host-staged gloo reduces synchronously: nothing to overlap)

    def hook(g):
        _start_range(flat, start, flat.grad.numel())
        return g

    t.register_hook(hook)


class _Anchor(torch.autograd.Function):
    """Identity on x whose backward runs once the gradient of every op that consumed x is
    complete -- i.e. after the whole sub-network x feeds: starts that network's gradient
    buckets then (x itself need not require grad; the anchor tensor does)."""

    @staticmethod
    def forward(ctx, x, anchor, flat, lo, hi):
        ctx.args = (flat, lo, hi)
        ctx.set_materialize_grads(False)  # gx is None when x's consumers skip it
        out = x.view_as(x)
        if not x.requires_grad:
            # the output requires grad only through the anchor: its consumers (the
            # posterior net's stem conv) compute no data gradient for it (ops._conv_bwd)
            out._vae2_no_dx = True
        return out

    @staticmethod
    def backward(ctx, gx, *_):
        flat, lo, hi = ctx.args
        _start_range(flat, lo, hi, own_stream=True)  # the network ran on this stream
        return gx, None, None, None, None


_ANCHOR = {}


def anchor_reduce(x, flat, lo=0, hi=None):
    """x, routed so that flat.grad[lo:hi] is all-reduced (async) as soon as the backward
    of the sub-network fed by x is done: the posterior net's buckets start while the
    encoder's backward still runs (its trunk is the deepest part of the step)."""
    if flat is None or not _overlap_ok() or not torch.is_grad_enabled():
        return x
    dev = x.device
    a = _ANCHOR.get(dev)
    if a is None:
        a = _ANCHOR[dev] = torch.zeros((), device=dev, requires_grad=True)
    return _Anchor.apply(x, a, flat, lo, flat.grad.numel() if hi is None else hi)


def allreduce_grads(flats, bucket_elems=BUCKET_ELEMS):
    """Mean-reduce the flat gradient buffers over all ranks (DDP semantics)."""
    if not is_dist():
        return
    streams.join_all()
    ws = world_size()
    pending = []
    for f in flats:
        g = f.grad
        done = sorted(_EARLY.pop(id(f), []), key=lambda e: (e[0], e[1]))
        works, gaps, pos = [], [], 0
        for lo, hi, w in done:  # the ranges no hook started yet
            if lo < pos:  # a range reduced twice would be scaled by the world size
                raise RuntimeError(f"overlapping early gradient buckets [{lo}, {hi}) "
                                   f"(previous range ends at {pos}): a second backward "
                                   "before allreduce_grads?")
            if lo > pos:
                gaps.append((pos, lo))
            pos = hi
            works += w
        if pos < g.numel():
            gaps.append((pos, g.numel()))
        for lo, hi in gaps:
            if dist.get_backend(grad_group()) == "gloo":
                bucket_allreduce(g[lo:hi], bucket_elems, group=grad_group())
            else:
                works += [dist.all_reduce(g[off:min(off + bucket_elems, hi)], group=grad_group(),
                                          async_op=True)
                          for off in range(lo, hi, bucket_elems)]
        pending.append((g, works))
    for g, works in pending:
        for w in works:
            w.wait()  # the compute stream waits for the bucket (no host sync)
        call("vae2_scale", ops.ptr(g), ops.ptr(g), g.numel(), 1.0 / ws, ops.stream_ptr())


_DDP_GUARD = False


def guard_ddp():
    """Make torch.nn.parallel.DistributedDataParallel refuse the HIP-path modules.

    The reference wraps FullModel_encdec / FullModel_D in DDP(find_unused_parameters=True)
    (/root/reference/tools/train.py:225-229).  Here the HIP backward kernels accumulate
    every parameter gradient into the flat main_grad buffers (vae2.params), so DDP's
    per-parameter gradient hooks never fire: it would all-reduce nothing and every rank
    would silently train on its own gradients.  Wrapping a module that contains a HIP-path
    network therefore raises, naming the replacement (allreduce_grads after backward).
    Installed once, on import of vae2.hrnet; other modules wrap as before."""
    global _DDP_GUARD
    if _DDP_GUARD:
        return
    from torch.nn.parallel import DistributedDataParallel as DDP
    orig = DDP.__init__

    def __init__(self, module, *args, **kwargs):
        hip = [type(m).__name__ for m in module.modules() if getattr(m, "_vae2_hip_module", False)]
        if hip:
            raise RuntimeError(
                f"DistributedDataParallel cannot wrap a HIP-path module ({hip[0]}): its "
                "parameter gradients are accumulated into flat main_grad buffers, so DDP's "
                "per-parameter hooks would never fire and no gradient would be all-reduced. "
                "Call vae2.dist.set_sync_bn(True) once and vae2.dist.allreduce_grads("
                "optimizer.flats) after backward() instead (INTEGRATION.md, 'The "
                "reference's own tools/train.py').")
        orig(self, module, *args, **kwargs)

    __init__.__wrapped__ = orig
    __init__.__doc__ = orig.__doc__
    DDP.__init__ = __init__
    _DDP_GUARD = True


def reduce_tensor(inp):
    """dist.reduce(sum) to rank 0 (function.py:32-43)."""
    if world_size() < 2:
        return inp
    with torch.no_grad():
        dist.reduce(inp, dst=0)
    return inp
