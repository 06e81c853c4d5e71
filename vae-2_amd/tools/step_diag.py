"""Host-issue vs device time of the bench step: is the step launch-bound?

    python vae-2_amd/tools/step_diag.py [--steps 5]

Prints, per phase (forward / backward / all-reduce+Adam), the host time spent
issuing work, and the wall time of whole steps with a device sync.  When the
host issue time of a step approaches its wall time, the GPU is starved by the
Python/launch path rather than by kernel speed.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, _p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    from helpers import build, make_cfg
    from vae2 import dist as vdist
    from vae2.model import FullModel_encdec
    from vae2.optim import FusedAdam
    dev = torch.device("cuda", 0)
    L, H, W, B = 3, 128, 256, a.batch
    ed, ez = build(make_cfg("w18", L=L, hw=(H, W)))
    fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(dev)
    fm.defer_checks = True
    opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-4)
    xs = [torch.randn(B, 3 * L, H, W, device=dev) for _ in range(3)]
    zc = ez.z_dim
    acc = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0, "host_step": 0.0, "wall_step": 0.0}

    def step(rec):
        t0 = time.perf_counter()
        opt.zero_grad()
        fm.set_noise(torch.randn(B, zc, 1, 1), torch.randn(B, zc, 1, 1))
        loss = fm(*xs, 1.0)[0][0]
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        vdist.allreduce_grads(opt.flats)
        opt.step()
        t3 = time.perf_counter()
        if rec:
            acc["fwd"] += t1 - t0
            acc["bwd"] += t2 - t1
            acc["opt"] += t3 - t2
            acc["host_step"] += t3 - t0

    for _ in range(3):
        step(False)
    torch.cuda.synchronize()
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step(True)
        torch.cuda.synchronize()
        acc["wall_step"] += time.perf_counter() - t0
    print({k: round(1e3 * v / a.steps, 2) for k, v in acc.items()}, "ms/step")
    # pipelined wall (no sync between steps), as bench.py times it
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print({"pipelined_host_ms": round(1e3 * (t1 - t0) / a.steps, 2),
           "pipelined_wall_ms": round(1e3 * (t2 - t0) / a.steps, 2)})
    from vae2.graph import StepGraph

    def full():
        opt.zero_grad()
        fm.set_noise(torch.randn(B, zc, 1, 1, device=dev), torch.randn(B, zc, 1, 1, device=dev))
        loss = fm(*xs, 1.0)[0][0]
        loss.backward()
        opt.step()
        return loss
    t0 = time.perf_counter()
    g = StepGraph(full, warmup=2)
    t1 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print({"graph_capture_s": round(t1 - t0, 2), "graph_nodes_first_replay_ms":
           round(1e3 * (t2 - t1), 2), "graph_replay_ms": round(1e3 * (t3 - t2) / a.steps, 2)})


if __name__ == "__main__":
    main()
