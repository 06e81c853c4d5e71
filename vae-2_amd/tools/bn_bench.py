"""Microbenchmark of the multi-layer BatchNorm kernels at the bench's lock-stepped
branch shapes (one HRNet depth level: 18/36/72/144 channels at 1, 1/2, 1/4, 1/8 of
128x256, 8 images).

    python vae-2_amd/tools/bn_bench.py [--iters 50] [--relu 1] [--res 1]

Times vae2_bn_multi_apply / _bwd_reduce / _bwd_apply with HIP events and prints the
algorithmic HBM rate (every tensor read or written once).
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from vae2 import _lib  # noqa: E402
from vae2._lib import call  # noqa: E402
from vae2.ops import _bn_layer, _empty, new_act, stream_ptr  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--relu", type=int, default=1)
    ap.add_argument("--res", type=int, default=1)
    ap.add_argument("--tune", default="", help="vae2_conv2d_set_tune key=value[,key=value]")
    ap.add_argument("--mask", type=int, default=0, help="ReLU mask bytes (residual layers)")
    ap.add_argument("--set", default="level", choices=["level", "narrow", "wide"],
                    help="level: 18/36/72/144 at 1, 1/2, 1/4, 1/8 of 128x256; narrow: the "
                         "18/36/72 launch; wide: one 64-channel layer at 128x256")
    ap.add_argument("--only", default="", help="comma list of passes (apply,bwd_reduce,bwd_apply)")
    a = ap.parse_args()
    lib = _lib.load()
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        lib.vae2_conv2d_set_tune(int(k), int(v))
    dev = torch.device("cuda")
    shapes = {"level": [(128, 256, 18), (64, 128, 36), (32, 64, 72), (16, 32, 144)],
              "narrow": [(128, 256, 18), (64, 128, 36), (32, 64, 72)],
              "wide": [(128, 256, 64)]}[a.set]
    lay = (_lib.BnLayer * len(shapes))()
    keep = []
    nbytes = {"apply": 0, "bwd_reduce": 0, "bwd_apply": 0}
    for i, (h, w, c) in enumerate(shapes):
        like = torch.empty(1, device=dev)
        x, y, r, dy, dx, dres = (new_act((a.n, h, w, c), like).normal_() for _ in range(6))
        save = torch.cat([torch.zeros(c), torch.ones(c), torch.ones(c), torch.zeros(c)]).to(dev)
        gamma = torch.ones(c, device=dev)
        rows = _lib.load().vae2_bn_partial_rows(ctypes.byref(_lib.Act(a.n, h, w, c, c)))
        part = _empty((2 * rows * c,), x)
        sums = torch.zeros(2 * c, dtype=torch.float64, device=dev)
        keep += [x, y, r, dy, dx, dres, save, gamma, part, sums]
        lay[i] = _bn_layer(x, r if a.res else None, y, dy, dres if a.res else None, save, gamma,
                           part, sums.data_ptr(), None, float(a.n * h * w), a.relu)
        if a.mask:  # ReLU mask bytes instead of y in the backward passes (residual layers)
            mk = torch.randint(0, 16, (a.n * h * w * ((c + 3) // 4),), dtype=torch.uint8, device=dev)
            keep.append(mk)
            lay[i].mask = mk.data_ptr()
        t = 4 * a.n * h * w * c
        nbytes["apply"] += t * (3 if a.res else 2)
        nbytes["bwd_reduce"] += t * (3 if a.res else 2)
        nbytes["bwd_apply"] += t * (4 + (1 if a.res else 0) + (1 if a.res else 0))
    s = stream_ptr()
    n = len(shapes)
    for name, fn in (("apply", lambda: call("vae2_bn_multi_apply", n, lay, s)),
                     ("bwd_reduce", lambda: call("vae2_bn_multi_bwd_reduce", n, lay, s)),
                     ("bwd_apply", lambda: call("vae2_bn_multi_bwd_apply", n, lay, s))):
        if a.only and name not in a.only.split(","):
            continue
        us = timeit(fn, a.iters)
        print(f"  {name:12s} {us:8.1f} us  {nbytes[name] / us / 1e3:8.1f} GB/s")


if __name__ == "__main__":
    main()
