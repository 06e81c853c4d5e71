"""The one-shot SyncBN peer all-reduce (csrc/syncbn.hip, vae2_syncbn_allreduce): 2 ranks
sharing the one MI355X of a test box exchange IPC handles over gloo and all-reduce float64
statistics buffers through each other's receive areas.  The result must be the exact
rank-order sum on both ranks (bit for bit), across hundreds of exchanges of varying size
(both receive slots reused many times), inside a replayed HIP graph (the exchange sequence
number lives in device memory), and with no timeout recorded.  Reports the latency per
exchange (same-device IPC; on 8 GPUs the peers are reached over xGMI)."""
import os
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dist_gpu import ROOT, _port

pytestmark = pytest.mark.gpu


def _work(rank, world, port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from vae2 import dist as vdist
    vdist.FORCE_IPC = True
    vdist.set_sync_bn(True)
    assert vdist.init_syncbn_ipc(dist.group.WORLD), "IPC exchange did not come up"
    gen = torch.Generator().manual_seed(100 + rank)
    sizes = [1, 7, 64, 650, 2048, 4096, 33, 1500] * 40
    ins = [torch.randn(n, generator=gen, dtype=torch.float64) for n in sizes]
    outs = []
    for x in ins:
        t = x.cuda()
        vdist.syncbn_all_reduce_(t)
        outs.append(t)
    torch.cuda.synchronize()
    got = [t.cpu() for t in outs]
    # exact reference: every rank's inputs, summed in rank order on the host
    allin = [None] * world
    dist.all_gather_object(allin, [x.numpy() for x in ins])
    ok = True
    for i in range(len(ins)):
        ref = torch.from_numpy(allin[0][i]).clone()
        for r in range(1, world):
            ref += torch.from_numpy(allin[r][i])
        ok &= torch.equal(got[i], ref)
    # issued from two streams in turn (the step's posterior net / past decoder side streams):
    # the exchanges still pair with the peers' same exchange (host issue order)
    streams2 = [torch.cuda.Stream(), torch.cuda.Stream()]
    ms = []
    for k in range(40):
        v = torch.full((300,), float((rank + 1) * (k + 1)), dtype=torch.float64, device="cuda")
        with torch.cuda.stream(streams2[k % 2]):
            vdist.syncbn_all_reduce_(v)
        ms.append(v)
    torch.cuda.synchronize()
    for k, v in enumerate(ms):
        ok &= bool((v.cpu() == sum((r + 1) * (k + 1) for r in range(world))).all())
    # inside a HIP graph: 6 exchanges captured, replayed 4 times (fresh inputs each time)
    bufs = [torch.zeros(512, dtype=torch.float64, device="cuda") for _ in range(6)]
    src = [torch.zeros(512, dtype=torch.float64, device="cuda") for _ in range(6)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up outside the capture (same call sequence)
        for b, s in zip(bufs, src):
            b.copy_(s)
            vdist.syncbn_all_reduce_(b)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for b, s in zip(bufs, src):
            b.copy_(s)
            vdist.syncbn_all_reduce_(b)
    gok = True
    for it in range(4):
        vals = [torch.full((512,), float(rank + 1) * (it + 1) + k, dtype=torch.float64) for k in range(6)]
        for s, v in zip(src, vals):
            s.copy_(v)
        g.replay()
        torch.cuda.synchronize()
        for k, b in enumerate(bufs):
            want = sum(float(r + 1) * (it + 1) + k for r in range(world))
            gok &= bool((b.cpu() == want).all())
    # latency inside a replayed graph (how the training step issues them): 6 exchanges of
    # 512 doubles + 6 copies per replay
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    torch.cuda.synchronize()
    us_graph = (time.perf_counter() - t0) / (200 * 6) * 1e6
    # latency: back-to-back exchanges of a depth level's statistics (2048 doubles)
    t = torch.randn(2048, dtype=torch.float64, device="cuda")
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500):
        vdist.syncbn_all_reduce_(t)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 500 * 1e6
    vdist.syncbn_check()
    q.put((rank, "ok", ok, gok, us, us_graph))
    dist.barrier()
    dist.destroy_process_group()


def _worker(rank, world, port, q):
    try:
        _work(rank, world, port, q)
    except BaseException:
        import traceback
        q.put((rank, "error", traceback.format_exc()))
        raise


@pytest.mark.timeout(300)
def test_syncbn_ipc_two_ranks_exact_sums():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    res, deadline = [], time.time() + 200
    while len(res) < 2:
        try:
            res.append(q.get(timeout=5))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail(f"IPC exchange run failed: exit codes {[p.exitcode for p in procs]}")
    for p in procs:
        p.join(timeout=60)
    errors = [r for r in res if r[1] == "error"]
    assert not errors, errors[0][2]
    for rank, _, ok, gok, us, usg in sorted(res):
        print(f"rank {rank}: exact {ok}, graph replay {gok}, {us:.1f} us per 2048-double exchange "
              f"(eager issue), {usg:.1f} us per exchange in a replayed graph")
        assert ok, "eager exchanges differ from the rank-order sums"
        assert gok, "graph-replayed exchanges wrong"


def _fail_work(rank, world, port, q):
    """Failure semantics of the exchange (ABI 12): a late peer and diverged exchange
    sequences fail loudly, stickily and with NaN statistics -- never a silent local sum."""
    import sys
    for p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from vae2 import dist as vdist
    vdist.FORCE_IPC = True
    vdist.set_sync_bn(True)
    out = {}
    # (1) a late peer: rank 1 arrives at exchange 2 after rank 0's bound (0.3 s) expired
    assert vdist.init_syncbn_ipc(dist.group.WORLD), "IPC exchange did not come up"
    vdist._SB.set_timeout(0.3)
    res = []
    for k in range(3):
        if k == 1 and rank == 1:
            time.sleep(1.5)
        t = torch.full((64,), float(rank + 1), dtype=torch.float64, device="cuda")
        vdist.syncbn_all_reduce_(t)
        torch.cuda.synchronize()
        res.append(t.cpu())
    out["late"] = [(bool(torch.isnan(r).all()), float(r[0])) for r in res]
    try:
        vdist.syncbn_check()
        out["late_raised"] = False
    except vdist.SyncBNExchangeError:
        out["late_raised"] = True
    dist.barrier()
    # (2) diverged sequences: same exchange number, different payload lengths
    assert vdist.init_syncbn_ipc(dist.group.WORLD), "second IPC comm did not come up"
    vdist._SB.set_timeout(5.0)
    t = torch.ones(10 + 2 * rank, dtype=torch.float64, device="cuda")
    vdist.syncbn_all_reduce_(t)
    torch.cuda.synchronize()
    out["mismatch_nan"] = bool(torch.isnan(t.cpu()).all())
    out["mismatch_err"] = vdist._SB.error()
    q.put((rank, "ok", out))
    dist.barrier()
    dist.destroy_process_group()


def _fail_worker(rank, world, port, q):
    try:
        _fail_work(rank, world, port, q)
    except BaseException:
        import traceback
        q.put((rank, "error", traceback.format_exc()))
        raise


@pytest.mark.timeout(300)
def test_syncbn_ipc_failures_are_sticky_and_nan():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    res, deadline = [], time.time() + 200
    while len(res) < 2:
        try:
            res.append(q.get(timeout=5))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail(f"IPC failure run failed: exit codes {[p.exitcode for p in procs]}")
    for p in procs:
        p.join(timeout=60)
    errors = [r for r in res if r[1] == "error"]
    assert not errors, errors[0][2]
    by = {r: o for r, _, o in res}
    print(by)
    # exchange 0: exact on both ranks
    assert by[0]["late"][0] == (False, 3.0) and by[1]["late"][0] == (False, 3.0)
    # rank 0 waited for rank 1 past its bound: NaN, then sticky NaN (no pairing with
    # rank 1's late exchange 1 as if it were its exchange 2)
    assert by[0]["late"][1][0] and by[0]["late"][2][0]
    # rank 1 found rank 0's exchange-1 payload (rank 0 stored it before waiting): exact; its
    # exchange 2 then waits for a rank that stopped raising flags: NaN
    assert by[1]["late"][1] == (False, 3.0) and by[1]["late"][2][0]
    assert by[0]["late_raised"] and by[1]["late_raised"]
    for r in (0, 1):
        assert by[r]["mismatch_nan"] and by[r]["mismatch_err"] != 0
