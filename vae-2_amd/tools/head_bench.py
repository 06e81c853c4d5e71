"""Microbenchmark of the per-branch head kernels at the bench shape (one head).

    python vae-2_amd/tools/head_bench.py [--n 8 --h 128 --w 256] [--iters 20]

Times each kernel of vae2/heads.py with HIP events on the current stream and prints
the average time and the algorithmic HBM rate (bytes each kernel must move once).
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from vae2 import _lib  # noqa: E402
from vae2._lib import Act, call  # noqa: E402
from vae2.ops import act_of, new_act, ptr, stream_ptr  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--h", type=int, default=128)
    ap.add_argument("--w", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma list of upsum,adj,out (profiling runs)")
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))

    def want(k):
        return not only or k in only
    lib = _lib.load()
    dev = torch.device("cuda")
    split = (18, 36, 72, 144)
    C = sum(split)
    n, H, W = a.n, a.h, a.w
    sizes = [(H, W)]
    for _ in split[1:]:
        sizes.append(((sizes[-1][0] + 1) // 2, (sizes[-1][1] + 1) // 2))
    ys = [new_act((n, h, w, c), torch.empty(1, device=dev)).normal_() for c, (h, w) in zip(split, sizes)]
    zs = [new_act((n, h, w, C), ys[0]).normal_() for (h, w) in sizes[1:]]
    P = n * H * W
    y = torch.empty(((C + 63) // 64) * P * 64, device=dev)  # B64 layout
    w = torch.randn(C, C, device=dev) * 0.05
    bias = torch.randn(C, device=dev)
    wp0 = torch.empty(lib.vae2_conv2d_packed_size(C, split[0], 1, 0), device=dev)
    call("vae2_conv2d_pack_weight_ld", ptr(w), C, split[0], 1, 0, C, ptr(wp0), stream_ptr())
    s = stream_ptr()
    x0p, x0a = act_of(ys[0])
    yp, ya = ptr(y), Act(n, H, W, C, C)
    rows = lib.vae2_conv1x1_upsum_stats_rows(ctypes.byref(ya))
    stats = torch.empty(2 * rows * C, device=dev)
    ups = (ctypes.c_void_p * 3)(*[act_of(z)[0] for z in zs])
    upds = (Act * 3)(*[act_of(z)[1] for z in zs])
    P = n * H * W
    res = []

    def upsum():
        call("vae2_conv1x1_upsum_fwd", x0p, ctypes.byref(x0a), ptr(wp0), ptr(bias), 3, ups, upds,
             yp, ctypes.byref(ya), ptr(stats), s)
    zb = sum(z.numel() for z in zs) * 4
    if want("upsum"):
        res.append(("upsum (y write + x0 + z read)", timeit(upsum, a.iters),
                    P * C * 4 + P * 20 * 4 + zb))
        lib.vae2_heads_set_algo(8)
        res.append(("  LDS-staged kernel (upsum_kernel)", timeit(upsum, a.iters),
                    P * C * 4 + P * 20 * 4 + zb))
        lib.vae2_heads_set_algo(8 | 2)
        res.append(("  same, 12 staging columns per source", timeit(upsum, a.iters),
                    P * C * 4 + P * 20 * 4 + zb))
        lib.vae2_heads_set_algo(0)

    gs = [new_act((n, h, w_, C), ys[0]) for (h, w_) in sizes[1:]]
    gptrs = (ctypes.c_void_p * 3)(*[act_of(g)[0] for g in gs])
    gacts = (Act * 3)(*[act_of(g)[1] for g in gs])
    lib.vae2_heads_set_algo(4)  # the two-pass form's workspace (the largest)
    usz = lib.vae2_upsample_bilinear_bwd_multi_ws_size(ctypes.byref(ya), 3, gacts)
    lib.vae2_heads_set_algo(0)
    uws = torch.empty(usz, device=dev)

    ynp, yna = act_of(new_act((n, H, W, C), ys[0]).normal_())

    def adj():
        call("vae2_upsample_bilinear_bwd_multi", ynp, ctypes.byref(yna), 3, gptrs, gacts, ptr(uws),
             usz, s)
    for algo, name in () if not want("adj") else ((0, "upsample adjoint x3, one pass (dy read + dx write)"),
                       (16 << 8, "  same, 16 dy rows per workgroup"),
                       (64 << 8, "  same, 64 dy rows per workgroup"),
                       (4, "  two-pass (horizontal -> hb -> vertical)"),
                       (5, "  two-pass, per-channel-lane vertical pass")):
        lib.vae2_heads_set_algo(algo)
        res.append((name, timeit(adj, a.iters), P * C * 4 + zb))
    lib.vae2_heads_set_algo(0)

    save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
    w2 = torch.randn(3, C, device=dev)
    b2 = torch.randn(3, device=dev)
    out = new_act((n, H, W, 3), ys[0])
    op, oa = act_of(out)

    def hfwd():
        call("vae2_head_out_fwd", yp, ctypes.byref(ya), ptr(save), ptr(w2), ptr(b2), 3, op,
             ctypes.byref(oa), s)
    if want("out"):
        res.append(("head_out_fwd (y read)", timeit(hfwd, a.iters), P * C * 4))

    wsz = lib.vae2_head_out_bwd_ws_size(ctypes.byref(ya), 3)
    ws = torch.empty(wsz, device=dev)
    sums = torch.zeros(2 * C, dtype=torch.float64, device=dev)
    dg, db, dw2, db2 = (torch.zeros(C, device=dev), torch.zeros(C, device=dev),
                        torch.zeros(3 * C, device=dev), torch.zeros(3, device=dev))

    def hred():
        call("vae2_head_out_bwd_reduce", yp, ctypes.byref(ya), ptr(save), ptr(w2), 3, op,
             ctypes.byref(oa), ptr(sums), ptr(dg), ptr(db), ptr(dw2), ptr(db2), ptr(ws), wsz, s)
    if want("out"):
        res.append(("head_out_bwd_reduce (y read)", timeit(hred, a.iters), P * C * 4))
        lib.vae2_heads_set_algo(16)
        res.append(("  same, 4 pixels in flight per thread", timeit(hred, a.iters), P * C * 4))
        lib.vae2_heads_set_algo(0)
    dy = new_act((n, H, W, C), ys[0])
    dyp, dya = act_of(dy)
    yn = new_act((n, H, W, C), ys[0])
    dbias = torch.zeros(C, device=dev)

    def happ():
        call("vae2_head_out_bwd_apply", yp, ctypes.byref(ya), ptr(save), ptr(dg), ptr(w2), 3, op,
             ctypes.byref(oa), ptr(sums), float(P), dyp, ctypes.byref(dya), ptr(dbias), ptr(ws),
             wsz, s)
    if want("out"):
        res.append(("head_out_bwd_apply (y read + dy write)", timeit(happ, a.iters),
                    2 * P * C * 4))
        lib.vae2_heads_set_algo(32)
        res.append(("  same, 4 pixels in flight per thread", timeit(happ, a.iters),
                    2 * P * C * 4))
        lib.vae2_heads_set_algo(0)

    def copy():
        dy.copy_(yn)
    if want("out"):
        res.append(("torch copy y->dy (reference rate)", timeit(copy, a.iters), 2 * P * C * 4))
    print(f"shape n={n} {H}x{W}, C={C}")
    for name, us, byts in res:
        print(f"  {name:45s} {us:9.1f} us  {byts / us / 1e3:8.1f} GB/s")


if __name__ == "__main__":
    main()
