"""Per-shape timing of the conv kernels (forward, data-grad, weight-grad) with HIP events.

    python tools/conv_bench.py [--batch 8] [--iters 20]

Shapes are the dominant ones of the 128x256 ELBO step; the
FLOP count is the algorithmic 2*M*N*K of each GEMM.
"""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))

import torch  # noqa: E402

from vae2 import _lib, ops  # noqa: E402
from vae2._lib import call  # noqa: E402

SHAPES = [  # H, W, Cin, Cout, k, stride, count per step (App. B, fwd)
    (128, 256, 64, 64, 3, 1, 12),
    (128, 256, 270, 270, 1, 1, 9),
    (128, 256, 64, 256, 1, 1, 12),
    (128, 256, 18, 18, 3, 1, 96),
    (64, 128, 36, 36, 3, 1, 96),
    (32, 64, 72, 72, 3, 1, 80),
    (16, 32, 144, 144, 3, 1, 32),
    (128, 256, 256, 18, 3, 1, 4),
    (128, 256, 256, 64, 1, 1, 4),
    (128, 256, 18, 36, 3, 2, 24),
]

# Every ELBO conv shape except the per-branch heads: input H, W.
ALL_SHAPES = [
    (128, 256, 18, 64, 3, 1, 1), (128, 256, 64, 64, 3, 1, 12), (128, 256, 64, 64, 1, 1, 4),
    (128, 256, 64, 256, 1, 1, 12), (128, 256, 256, 64, 1, 1, 4), (128, 256, 256, 18, 3, 1, 4),
    (128, 256, 256, 36, 3, 2, 4), (128, 256, 18, 18, 3, 1, 96), (128, 256, 18, 36, 3, 2, 24),
    (128, 256, 18, 18, 3, 2, 28), (128, 256, 9, 64, 3, 1, 3), (128, 256, 38, 18, 3, 1, 1),
    (128, 256, 28, 18, 3, 1, 2), (64, 128, 36, 36, 3, 1, 96), (64, 128, 36, 18, 1, 1, 24),
    (64, 128, 36, 72, 3, 2, 24), (64, 128, 18, 72, 3, 2, 20), (64, 128, 18, 18, 3, 2, 8),
    (64, 128, 36, 36, 3, 2, 8), (64, 128, 56, 36, 3, 1, 1), (64, 128, 46, 36, 3, 1, 2),
    (32, 64, 72, 72, 3, 1, 80), (32, 64, 72, 18, 1, 1, 20), (32, 64, 72, 36, 1, 1, 20),
    (32, 64, 72, 144, 3, 2, 12), (32, 64, 18, 144, 3, 2, 8), (32, 64, 36, 144, 3, 2, 8),
    (32, 64, 92, 72, 3, 1, 1), (32, 64, 82, 72, 3, 1, 2), (16, 32, 144, 144, 3, 1, 32),
    (16, 32, 144, 18, 1, 1, 8), (16, 32, 144, 36, 1, 1, 8), (16, 32, 144, 72, 1, 1, 8),
    (16, 32, 164, 144, 3, 1, 1), (16, 32, 154, 144, 3, 1, 2),
]


def timeit(fn, iters):
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    if os.environ.get("VAE2_LIB"):  # A/B runs against another build of the library
        _lib.LIB_PATH = os.environ["VAE2_LIB"]
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", type=int, nargs="*", help="indices into SHAPES")
    ap.add_argument("--algo", type=int, nargs="*", default=[0],
                    help="vae2_conv2d_set_algo values to compare (0 auto, 1 gather, 2 direct)")
    ap.add_argument("--all", action="store_true", help="every ELBO conv shape (ALL_SHAPES)")
    ap.add_argument("--bf16", action="store_true", help="bf16 MFMA operands")
    ap.add_argument("--tune", default="", help="vae2_conv2d_set_tune key=value[,key=value]")
    a = ap.parse_args()
    if a.all:
        SHAPES[:] = ALL_SHAPES
    lib = _lib.load()
    warm = torch.randn(4096, 4096, device="cuda")
    for _ in range(200):  # bring the clocks up before the first timed shape
        warm = warm @ warm.T * 1e-4
    torch.cuda.synchronize()
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        if lib.vae2_conv2d_set_tune(int(k), int(v)) < 0:
            raise SystemExit(f"unknown conv tune key {k}")
    for algo in a.algo:
        lib.vae2_conv2d_set_algo(algo)
        lib.vae2_conv2d_set_mfma_bf16(1 if a.bf16 else 0)
        print(f"== algo {algo}")
        run(a, lib)


def run(a, lib):
    dev = "cuda"
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    rows = []
    print(f"{'shape':34s} {'fwd us':>8s} {'TF/s':>6s} {'dgrad us':>9s} {'TF/s':>6s} "
          f"{'wgrad us':>9s} {'TF/s':>6s}")
    for idx, (H, W, ci, co, k, st, cnt) in enumerate(SHAPES):
        if a.only and idx not in a.only:
            continue
        B = a.batch
        x = ops.new_act((B, H, W, ci), torch.empty(1, device=dev))
        x.normal_()
        oh, ow = (H + 2 * (k // 2) - k) // st + 1, (W + 2 * (k // 2) - k) // st + 1
        w = torch.randn(co, ci, k, k, device=dev) * 0.05
        y = ops.new_act((B, oh, ow, co), x)
        dy = ops.new_act((B, oh, ow, co), x)
        dy.normal_()
        dx = ops.new_act((B, H, W, ci), x)
        dw = torch.zeros_like(w)
        wp0 = ops.packed_weight(w, 0)
        wp1 = ops.packed_weight(w, 1)
        xp, xa = ops.act_of(x)
        yp, ya = ops.act_of(y)
        dyp, dya = ops.act_of(dy)
        dxp, dxa = ops.act_of(dx)
        pad = k // 2
        size = lib.vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xa), ctypes.byref(dya), k)
        ws = torch.empty(size, device=dev)
        s = ops.stream_ptr()
        flops = 2.0 * B * oh * ow * co * ci * k * k

        def fwd():
            call("vae2_conv2d_fwd", xp, ctypes.byref(xa), ops.ptr(wp0), None, yp,
                 ctypes.byref(ya), k, st, pad, 0.0, None, s)

        def dgrad():
            call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dya), ops.ptr(wp1), dxp,
                 ctypes.byref(dxa), k, st, pad, 0.0, s)

        def wgrad():
            call("vae2_conv2d_bwd_weight", xp, ctypes.byref(xa), dyp, ctypes.byref(dya),
                 ops.ptr(dw), None, k, st, pad, 0, ops.ptr(ws), size, s)

        tf, td, tw = timeit(fwd, a.iters), timeit(dgrad, a.iters), timeit(wgrad, a.iters)
        tot["fwd"] += tf * cnt
        tot["dgrad"] += td * cnt
        tot["wgrad"] += tw * cnt
        name = f"{H}x{W} {ci}->{co} k{k}s{st} x{cnt}"
        print(f"{name:34s} {tf:8.1f} {flops / tf / 1e6:6.1f} {td:9.1f} {flops / td / 1e6:6.1f} "
              f"{tw:9.1f} {flops / tw / 1e6:6.1f}", flush=True)
        rows.append((cnt * (tf + td + tw) / 1e3, cnt * tf / 1e3, cnt * td / 1e3, cnt * tw / 1e3, name))
    print("per-step ms by shape (total, fwd, dgrad, wgrad):")
    for r in sorted(rows, reverse=True):
        print(f"  {r[4]:34s} {r[0]:7.2f} {r[1]:7.2f} {r[2]:7.2f} {r[3]:7.2f}")
    print("weighted per-step ms (listed shapes only):",
          {k_: round(v / 1e3, 2) for k_, v in tot.items()})


if __name__ == "__main__":
    main()
