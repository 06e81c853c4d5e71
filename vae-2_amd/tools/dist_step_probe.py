"""Probe: eager distributed training steps through a world-size-1 RCCL group with the
distributed code paths forced on (vae2.dist.FORCE), W18 at 64x128 B=2 -- every SyncBN
exchange, the decoder-tail and posterior-net early buckets and the gradient buckets as
real RCCL collectives.  Prints one line per step (run it under `timeout`).

    python tools/dist_step_probe.py [--steps 3] [--graph]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--graph", action="store_true", help="capture the step and replay it")
    ap.add_argument("--capture-mode", default=None, choices=("global", "thread_local", "relaxed"))
    ap.add_argument("--dump-after", type=float, default=0,
                    help="print every thread's Python stack every N s (hang diagnosis)")
    a = ap.parse_args()
    if a.dump_after > 0:
        import faulthandler
        faulthandler.dump_traceback_later(a.dump_after, repeat=True, exit=False)
    from helpers import build, make_cfg
    from vae2 import dist as vdist
    from vae2.model import FullModel_encdec
    from vae2.optim import FusedAdam
    torch.cuda.set_device(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    from vae2.dist import prepare_nccl_env
    prepare_nccl_env()
    dist.init_process_group("nccl", rank=0, world_size=1)
    vdist.FORCE = True
    vdist.set_sync_bn(True)
    hw, B = (64, 128), 2
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(B, 9, *hw, generator=g).cuda() for _ in range(3)]
    eps = torch.randn(B, 10, 1, 1, generator=g).cuda()
    code = torch.randn(B, 10, 1, 1, generator=g).cuda()

    def make():
        ed, ez = build(make_cfg("w18", hw=hw))
        fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).cuda()
        fm.train()
        fm.defer_checks = True
        opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-3)

        def step():
            opt.zero_grad()
            fm.set_noise(eps, code)
            loss = fm(*xs, 1.0)[0][0]
            loss.backward()
            vdist.allreduce_grads(opt.flats)
            opt.step()
            return loss
        return step

    warm = 2
    ref = []
    if a.graph:  # eager reference: the warm-up steps + the replayed ones
        step = make()
        for i in range(warm + a.steps):
            ref.append(float(step()))
        print("eager", [round(v, 4) for v in ref], flush=True)
    run = make()
    if a.graph:
        from vae2.graph import StepGraph
        print("capturing", flush=True)
        run = StepGraph(run, warmup=warm, capture_error_mode=a.capture_mode).replay
        print("captured", flush=True)
    same = True
    for i in range(a.steps):
        t0 = time.time()
        loss = float(run())
        torch.cuda.synchronize()
        if ref:
            same &= loss == ref[warm + i]
        print(f"step {i}: loss {loss:.6f} ({time.time() - t0:.2f} s)"
              + (f" eager {ref[warm + i]:.6f}" if ref else ""), flush=True)
    if ref:
        print("graph == eager:", same, flush=True)
    dist.destroy_process_group()
    print("probe ok", flush=True)


if __name__ == "__main__":
    main()
