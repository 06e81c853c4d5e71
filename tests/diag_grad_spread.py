"""Diagnostic (not collected by pytest): spread of the HIP end-to-end gradients
against the fp64 oracle, per conv algorithm, next to the reference's own fp32
spread.  python tests/diag_grad_spread.py"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "vae-2_amd")):
    sys.path.insert(0, p)

from helpers import golden, rel, t  # noqa: E402
from test_model_gpu import CASES, DEV, hip_model, noise, oracle_grads  # noqa: E402


def main():
    from vae2 import _lib
    g = golden("tiny_native")
    g64 = oracle_grads(g, torch.float64)
    lib = _lib.load()
    grads = {}
    for algo in (1, 2):
        lib.vae2_conv2d_set_algo(algo)
        fm = hip_model(CASES["tiny_native"])
        from vae2.optim import FusedAdam
        opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-4)
        xt, x2t, x3t = (t(g[k]).to(DEV) for k in ("xt", "x2t", "x3t"))
        fm.set_noise(*noise(g, False))
        opt.zero_grad()
        fm(xt, x2t, x3t, 1.0)[0][0].backward()
        params = list(fm.encz_model.named_parameters(prefix="encz")) + \
            list(fm.encdec_model.named_parameters(prefix="ed"))
        grads[algo] = {n: p.main_grad.detach().cpu().clone() for n, p in params}
    names = list(grads[1])
    ref_norms = g["grad_norms"]
    floor = 1e-6 * ref_norms.max()
    rows = []
    for n, rn in zip(names, ref_norms):
        if rn <= floor:
            continue
        b = rel(t(g["grad/" + n]), g64[n])
        a1 = rel(grads[1][n], g64[n])
        a2 = rel(grads[2][n], g64[n])
        d12 = rel(grads[1][n], grads[2][n])
        rows.append((n, b, a1, a2, d12))
    arr = np.array([[r[1], r[2], r[3], r[4]] for r in rows])
    print("median ref32 / algo1 / algo2 / algo1-vs-2:", np.median(arr, 0))
    den = np.maximum(arr[:, 0], np.median(arr[:, 0]))
    print("max ratio vs max(ref, median ref): algo1", (arr[:, 1] / den).max(), " algo2",
          (arr[:, 2] / den).max())
    worst = sorted(rows, key=lambda r: -(r[3] / max(r[1], 1e-12)))[:8]
    for r in worst:
        print(f"  {r[0]:50s} ref {r[1]:.2e} a1 {r[2]:.2e} a2 {r[3]:.2e} a1-a2 {r[4]:.2e}")
    worst = sorted(rows, key=lambda r: -(r[2] / max(r[1], 1e-12)))[:5]
    for r in worst:
        print(f"  a1-worst {r[0]:50s} ref {r[1]:.2e} a1 {r[2]:.2e} a2 {r[3]:.2e}")


if __name__ == "__main__":
    main()
