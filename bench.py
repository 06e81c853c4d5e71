"""Benchmark: VAE² ELBO training step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], the metric's config): HRNet-W18-small-v2
encoder + two decoders + posterior net, 128x256 clips of 3 x CLIP_LENGTH=3 = 9
frames, 8 clips per GPU (weak scaling; 64 clips at 8 GPUs), fp32, random-init
weights (seed 0, the reference's init), synthetic Gaussian clips resident in HBM.
One step = posterior net + reparameterisation + encoder + 2 decoders forward,
L1 x3 + KL, backward, RCCL gradient all-reduce (N > 1, SyncBN statistics),
Adam.  frames/s = clips * 9 / step time, whole job.  At N=1 the step is
captured once as a HIP graph (vae2.graph.StepGraph: same kernels, one launch,
bit-identical to eager steps — tests/test_graph_gpu.py) and replayed; the noise
is drawn on the device inside the step so every replay samples fresh noise.

Printed JSON also carries:
  roofline      the dominant conv kernel (the igemm instantiation that runs the
                64->64 3x3 full-resolution convs), timed live with HIP events
                around its launches during --roofline-steps extra steps that follow
                the timed region (each timed launch isolated from the side streams,
                so the span is the kernel's own execution, as rocprof measures it);
                achieved = algorithmic FLOPs per launch / average launch time,
                against the fp32 matrix peak (157.3 TFLOP/s, MI355X_MICROARCH.md);
                traffic = HBM bytes per launch from the committed PMC measurement.
  cpu_baseline  the CPU oracle (oracle/ref_cpu.py, the reference's ops on CPU)
                timed on this host's cores, rank 0 at N=1 only, on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TF = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="clips per GPU")
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--clip-length", type=int, default=3)
    ap.add_argument("--arch", default="w18")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=2)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-steps", type=int, default=3)
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay the step as one captured HIP graph (auto: at N=1)")
    return ap.parse_args()


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC measurement
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this benchmark), else None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("kernel") == kernel.replace("void ", ""):
            best = d
    return best


def cpu_baseline(args):
    """Oracle ELBO step (fwd + bwd + torch Adam) on the host CPU, bounded sample."""
    from helpers import build, make_cfg
    from oracle import ref_cpu
    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    L, H, W, B = args.clip_length, args.height, args.width, args.cpu_batch
    ed, ez = build(make_cfg(args.arch, L=L, hw=(H, W)))
    params = list(ez.parameters()) + list(ed.parameters())
    opt = torch.optim.Adam(params, lr=1e-4)
    g = torch.Generator().manual_seed(1)
    xs = [torch.randn(B, 3 * L, H, W, generator=g) for _ in range(3)]

    def step():
        opt.zero_grad()
        e = torch.randn(B, ez.z_dim, 1, 1)
        c = torch.randn(B, ez.z_dim, 1, 1)
        terms, _, _ = ref_cpu.elbo(ez, ed, *xs, e, c)
        terms["loss_all"].backward()
        opt.step()

    step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        step()
    dt = (time.perf_counter() - t0) / args.cpu_steps
    return {"value": round(B * 3 * L / dt, 3), "unit": "frames/s", "cores": cores,
            "kind": "port",
            "sample": f"oracle/ref_cpu.py ELBO step fwd+bwd+Adam, {args.arch} {H}x{W}, "
                      f"{B} clips x {3 * L} frames, fp32, 1 warm-up + {args.cpu_steps} timed "
                      f"steps ({dt:.2f} s/step), torch CPU threads={cores}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from helpers import build, make_cfg
    from vae2 import dist as vdist
    from vae2 import prof
    from vae2.model import FullModel_encdec
    from vae2.optim import FusedAdam
    vdist.set_sync_bn(True)

    L, H, W, B = args.clip_length, args.height, args.width, args.batch
    ed, ez = build(make_cfg(args.arch, L=L, hw=(H, W)))
    fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(dev)
    fm.train()
    fm.defer_checks = True
    opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-4)
    if world > 1:
        for f in opt.flats:
            dist.broadcast(f.data, src=0)
    g = torch.Generator().manual_seed(1 + rank)
    xs = [torch.randn(B, 3 * L, H, W, generator=g).to(dev) for _ in range(3)]
    zc = ez.z_dim

    def eager_step():
        opt.zero_grad()
        fm.set_noise(torch.randn(B, zc, 1, 1, device=dev), torch.randn(B, zc, 1, 1, device=dev))
        losses = fm(*xs, 1.0)[0]
        losses[0].backward()
        vdist.allreduce_grads(opt.flats)
        opt.step()
        return losses[0]

    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1)
    step = eager_step
    if use_graph:
        from vae2.graph import StepGraph
        graph = StepGraph(eager_step, warmup=2)
        step = graph.replay
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    fm.check_anomalies()

    # ---- timed region: the metric (full stream concurrency, no instrumentation) ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    fm.check_anomalies()
    last_loss = float(loss)

    # ---- roofline phase: the same step, the dominant kernel's launches timed with
    # HIP events on their stream, each launch isolated from the side streams ----
    from vae2 import _lib
    kname = prof.fwd_kernel_name(_lib.Act(B, H, W, 64, 64), (B, H, W, 64), 3, 1, 1)
    timer = prof.KernelTimer(kname)
    if not args.no_roofline and args.roofline_steps > 0:
        torch.cuda.synchronize()
        with timer:
            for _ in range(args.roofline_steps):
                eager_step()
        torch.cuda.synchronize()
        fm.check_anomalies()

    if rank == 0:
        ms = 1e3 * elapsed / args.steps
        frames = world * B * 3 * L * args.steps
        out = {
            "metric": "training frames/sec on 128x256 8-frame Cityscapes clips, 1/2/4/8 MI355X",
            "value": round(frames / elapsed, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (Gaussian Cityscapes-shaped clips resident in HBM; random-init "
                    "weights, reference init seed 0)",
            "config": {"workload": f"VAE2 ELBO step (encz + encoder + 2 decoders fwd/bwd + "
                                   f"Adam), HRNet-{args.arch}-small-v2, {H}x{W}, "
                                   f"{B} clips/GPU x {3 * L} frames (CLIP_LENGTH={L})",
                       "global_batch": world * B, "frames_per_clip": 3 * L,
                       "image": [H, W], "parallelism": f"dp{world}",
                       "sync_bn": world > 1,
                       "launch": "hip_graph" if use_graph else "eager"},
            "last_loss": last_loss,
        }
        summ = timer.summary() if not args.no_roofline else None
        if summ:
            tr = pmc_traffic(kname)
            out["roofline"] = {"bound": "mfma", "kernel": kname,
                               "achieved": round(summ["tflops"], 3), "peak": FP32_MFMA_PEAK_TF,
                               "unit": "TFLOP/s",
                               "frac": round(summ["tflops"] / FP32_MFMA_PEAK_TF, 4),
                               "traffic": round(tr["hbm_bytes_per_launch"]) if tr else None,
                               "traffic_unit": "bytes/launch (PMC)",
                               "avg_launch_us": round(summ["avg_us"], 2),
                               "flops_per_launch": summ["flops_per_launch"],
                               "algorithmic_bytes_per_launch": summ["bytes_per_launch"],
                               "launches": summ["launches"],
                               "measured": f"{args.roofline_steps} steps after the timed region, "
                                           "launches isolated from side streams (eager)"}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
