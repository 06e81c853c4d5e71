"""Diagnostic (GPU): per-element accuracy of the conv kernels' forward / data gradient
against fp64 at given shapes, per algo (1 gather, 2 direct, +16 no VALU remainder):
max error, mean error (bias), and where the largest errors sit.
    python scripts/diag_dgrad.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.nn.grad import conv2d_input  # noqa: E402

DEV = "cuda"


def main():
    from vae2 import _lib, ops
    lib = _lib.load()
    for (n, h, w, cin, cout) in [(8, 32, 64, 72, 72), (2, 32, 64, 72, 72), (8, 64, 128, 36, 36),
                                 (8, 128, 256, 18, 18)]:
        g = torch.Generator().manual_seed(3)
        x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
        dy = torch.randn(n, cout, h, w, generator=g, dtype=torch.float64)
        wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) / (9 * cin) ** 0.5
        y64 = F.conv2d(x, wt, None, 1, 1)
        dx64 = conv2d_input((n, cin, h, w), wt, dy, 1, 1)
        for algo in (1, 2, 18):
            prev = lib.vae2_conv2d_set_algo(algo)
            try:
                xg = ops.new_act((n, h, w, cin), torch.empty(1, device=DEV))
                dyg = ops.new_act((n, h, w, cout), xg)
                with torch.no_grad():
                    xg.copy_(x.float().permute(0, 2, 3, 1).to(DEV))
                    dyg.copy_(dy.float().permute(0, 2, 3, 1).to(DEV))
                wg = wt.float().to(DEV)
                yg = ops.new_act((n, h, w, cout), xg)
                dxg = ops.new_act((n, h, w, cin), xg)
                xp, xa = ops.act_of(xg)
                yp, ya = ops.act_of(yg)
                dyp, dya = ops.act_of(dyg)
                dxp, dxa = ops.act_of(dxg)
                ops.call("vae2_conv2d_fwd", xp, ctypes.byref(xa), ops.ptr(ops.packed_weight(wg, 0)),
                         None, yp, ctypes.byref(ya), 3, 1, 1, 0.0, None, ops.stream_ptr())
                ops.call("vae2_conv2d_bwd_data", dyp, ctypes.byref(dya),
                         ops.ptr(ops.packed_weight(wg, 1)), dxp, ctypes.byref(dxa), 3, 1, 1, 0.0,
                         ops.stream_ptr())
                torch.cuda.synchronize()
            finally:
                lib.vae2_conv2d_set_algo(prev)
            for tag, got, ref in (("fwd", yg, y64), ("dgrad", dxg, dx64)):
                e = got.permute(0, 3, 1, 2).double().cpu() - ref
                scale = ref.abs().max()
                chan = e.abs().amax((0, 2, 3))
                worst = torch.nonzero(e.abs() == e.abs().max())[0].tolist()
                rows = e.abs().amax((0, 1, 3))
                cols = e.abs().amax((0, 1, 2))
                print(f"{n}x{h}x{w} {cin}->{cout} algo {algo:2d} {tag:5s}: max {float(e.abs().max() / scale):.2e} "
                      f"mean {float(e.mean() / scale):+.2e} rel-L2 {float(e.norm() / ref.norm()):.2e} "
                      f"worst(n,c,h,w) {worst} worst-chan {int(chan.argmax())} "
                      f"row-max/median {float(rows.max() / rows.median()):.1f} "
                      f"col-max/median {float(cols.max() / cols.median()):.1f}", flush=True)


if __name__ == "__main__":
    main()
