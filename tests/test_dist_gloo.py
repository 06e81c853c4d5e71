"""Data-parallel path on CPU: world size 2 over gloo (multi-GPU runs are the
driver's).  Covers the SyncBN statistics exchange, the bucketed gradient
all-reduce, and the invariant the reference's SyncBN + DDP setup guarantees
(SURVEY.md §4): N ranks x B/N clips == 1 rank x B clips, checked against the
reference's own golden vectors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys
    for p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)


def _w_stats(rank, world, port, q):
    _init(rank, world, port)
    from vae2 import ops
    local = torch.arange(6, dtype=torch.float64) * (rank + 1)
    out, count = ops._all_reduce_sums(local, 10.0, dist.group.WORLD)
    q.put((rank, out.tolist(), count))
    dist.destroy_process_group()


def _w_bucket(rank, world, port, q):
    _init(rank, world, port)
    from vae2 import dist as vdist
    buf = torch.full((1000,), float(rank + 1))
    vdist.bucket_allreduce(buf, bucket_elems=128)
    q.put((rank, float(buf.min()), float(buf.max())))
    dist.destroy_process_group()


def _w_invariant(rank, world, port, q):
    _init(rank, world, port)
    from helpers import build, golden, make_cfg, t
    from oracle import ref_cpu
    g = golden("tiny_native")
    ed, ez = build(make_cfg("tiny"))
    sl = slice(rank, rank + 1)  # one clip per rank
    ref_cpu.SYNC_GROUP = dist.group.WORLD
    terms, preds, _ = ref_cpu.elbo(ez, ed, t(g["xt"])[sl], t(g["x2t"])[sl], t(g["x3t"])[sl],
                                   t(g["eps"])[sl], t(g["code"])[sl])
    loss = terms["loss_all"].detach().clone()
    dist.all_reduce(loss)
    q.put((rank, float(loss) / world, [p.detach()[0].numpy() for p in preds]))
    dist.destroy_process_group()


def _w_ddp_guard(rank, world, port, q):
    """The reference's train.py:225-229 call on a HIP-path model: DDP must refuse it (its
    per-parameter hooks never fire: gradients go to main_grad); a plain module still wraps."""
    _init(rank, world, port)
    from helpers import build, make_cfg
    from vae2.model import FullModel_encdec
    from vae2.criterion import KLLoss, L1Loss
    ed, ez = build(make_cfg("tiny"))
    fm = FullModel_encdec(ez, ed, None, None, L1Loss(), KLLoss(), None, 1.0, 0.1, 1.0, 0.0)
    msg = None
    try:
        torch.nn.parallel.DistributedDataParallel(fm, find_unused_parameters=True)
    except RuntimeError as e:
        msg = str(e)
    plain = torch.nn.parallel.DistributedDataParallel(torch.nn.Linear(3, 2))
    q.put((rank, msg, type(plain).__name__))
    dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_sync_bn_sums_gloo():
    res = _run(_w_stats)
    for _, out, count in res:
        assert out == [3.0 * i for i in range(6)]
        assert count == 20.0


def test_bucketed_grad_allreduce_gloo():
    for _, lo, hi in _run(_w_bucket):
        assert lo == hi == 3.0


@pytest.mark.timeout(600)
def test_two_ranks_equal_one_rank_with_sync_bn():
    """2 ranks x 1 clip with SyncBN == the reference's 1 rank x 2 clips (golden)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import golden
    g = golden("tiny_native")
    res = _run(_w_invariant)
    for _, loss, _ in res:
        assert abs(loss - float(g["loss_loss_all"])) <= 1e-5 * abs(float(g["loss_loss_all"]))
    for rank, _, preds in res:
        np.testing.assert_allclose(preds[1], g["x2p"][rank], rtol=0, atol=1e-4 * np.abs(g["x2p"]).max())


def test_decoder_tail_range_is_the_decoders():
    """The early gradient buckets (vae2.dist.early_reduce_hook) cover exactly the
    trailing decf_* / decp_* parameters of the encoder-decoder's flat buffer."""
    from helpers import build, make_cfg
    from vae2 import dist as vdist
    from vae2.params import flatten
    ed, _ = build(make_cfg("tiny"))
    flat = flatten(ed)
    start = vdist.tail_range(flat)
    assert start is not None and 0 < start < flat.numel
    names = [n for n, o in zip(flat.names, flat.offsets) if o >= start]
    assert names and all(n.startswith(("decf_", "decp_")) for n in names)
    assert not any(n.startswith(("decf_", "decp_")) for n, o in zip(flat.names, flat.offsets)
                   if o < start)


def test_ddp_refuses_hip_path_model():
    """A reference caller that keeps DistributedDataParallel gets a clear error instead of
    silently un-reduced gradients (vae2.dist.guard_ddp); other modules are unaffected."""
    for _, msg, plain in _run(_w_ddp_guard):
        assert msg is not None and "allreduce_grads" in msg and "main_grad" in msg
        assert plain == "DistributedDataParallel"


class _TimedOutExchange:
    """Test double of vae2.dist.IpcExchange (csrc/syncbn.hip semantics) over gloo: exchange
    number `fail_at` times out on every rank (as when a third rank never arrived: the
    peers that did arrive all hit the kernel's bounded wait), and the comm stays failed --
    that exchange and every later one write NaN and exchange nothing; error() is nonzero."""

    def __init__(self, fail_at):
        self.fail_at, self.n, self.err = fail_at, 0, 0

    def takes(self, t, group=None):
        return t.dtype == torch.float64

    def all_reduce_(self, t):
        self.n += 1
        if self.n == self.fail_at:
            self.err = 1
        if self.err:
            t.fill_(float("nan"))
            return
        dist.all_reduce(t)

    def error(self):
        return self.err


class _StubBN(torch.nn.Module):
    """A SyncBatchNorm-shaped consumer of the exchange: global mean / variance of its input
    from (sum x, sum x^2) all-reduced through vae2.dist, then a scaled squared error."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.ones(()))

    def forward(self, xt, x2t, x3t, multiplier, is_baseline=False, baseline_mode=None):
        from vae2 import ops
        from vae2 import dist as vdist
        s = torch.stack([xt.sum(), (xt * xt).sum()]).double()
        s, count = ops._all_reduce_sums(s, float(xt.numel()), vdist.sync_bn_group())
        mean = (s[0] / count).float()
        var = (s[1] / count).float() - mean * mean
        loss = self.w * ((xt - mean) ** 2).mean() / var
        return [loss, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0], xt, x2t, x3t


def _w_dropped_exchange(rank, world, port, q):
    """adversarial_train over a stub SyncBN model whose 3rd statistics exchange times out:
    the loop must raise vae2.dist.SyncBNExchangeError at its next PRINT_FREQ point, with
    NaN statistics (not plausible local ones) in the step that lost the exchange."""
    _init(rank, world, port)
    from types import SimpleNamespace
    from vae2 import dist as vdist
    from vae2.trainer import NullWriter, adversarial_train
    vdist.set_sync_bn(True)
    vdist._SB = _TimedOutExchange(fail_at=3)
    model = _StubBN()
    losses = []
    orig_fwd = model.forward

    def fwd(*a, **k):
        out = orig_fwd(*a, **k)
        losses.append(float(out[0][0]))
        return out
    model.forward = fwd

    class Opt:
        flats = []

        def zero_grad(self):
            model.w.grad = None

        def step(self):
            pass
    gen = torch.Generator().manual_seed(rank)
    loader = [([torch.randn(2, 9, 4, 4, generator=gen) for _ in range(3)], "c")
              for _ in range(8)]
    cfg = SimpleNamespace(PRINT_FREQ=2)
    err = None
    try:
        adversarial_train(cfg, 0, 1, len(loader), 1e-4, len(loader), loader, Opt(), None, model,
                          None, {"writer": NullWriter(), "train_global_steps": 0}, "cpu", "/tmp",
                          use_multiplier=False)
    except vdist.SyncBNExchangeError as e:
        err = str(e)
    vdist._SB = None
    q.put((rank, err, losses))
    dist.destroy_process_group()


def test_timed_out_syncbn_exchange_raises_from_training_loop():
    """A SyncBN exchange that times out (IPC kernel semantics: sticky error word, NaN
    statistics) stops training at the trainer's next PRINT_FREQ check on every rank,
    instead of training on with wrong statistics (ADVICE r5 / VERDICT r5 item 1)."""
    for _, err, losses in _run(_w_dropped_exchange):
        assert err is not None and "timed out" in err
        # iterations 0, 1 exchanged normally; iteration 2 lost its exchange (NaN loss) and
        # the check at i_iter = 2 (PRINT_FREQ 2) raised before iteration 3 began
        assert len(losses) == 3
        assert all(np.isfinite(losses[:2])) and np.isnan(losses[2])
