"""Diagnostic: per-tensor gradient distances of one ELBO golden mode case (HIP vs fp64
oracle, fp32 reference vs fp64), and the fp64 oracle's own sensitivity to a 1e-7
relative perturbation of the inputs (how chaotic each tensor's gradient is).
    python scripts/diag_modes.py tiny_det"""
import os
import sys

import numpy as np
import torch

_root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_root, "tests"), os.path.join(_root, "vae-2_amd"), _root]
import vae2._lib as _L  # noqa: E402
_L.LIB_PATH = os.environ.get("VAE2_LIB", _L.LIB_PATH)
import test_model_gpu as tm  # noqa: E402
from helpers import rel  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "tiny_det"
spec = tm.MODE_CASES[case]
kw = spec["kw"]
g = tm.golden(case)
fm = tm.hip_model(kw)
det = kw.get("mode") == "DETERMINISTIC"
if not det:
    fm.set_noise(tm.t(g["eps"]), tm.t(g["code"]))
losses, *_ = fm(tm.t(g["xt"]).to(tm.DEV), tm.t(g["x2t"]).to(tm.DEV), tm.t(g["x3t"]).to(tm.DEV),
                spec.get("multiplier", 1.0), is_baseline=kw.get("baseline", False),
                baseline_mode=kw.get("mode", "VAE_NATIVE"),
                sampling_mode="prior_sampling" if spec.get("prior") else "default")
from vae2.params import flatten  # noqa: E402
for m in (fm.encz_model, fm.encdec_model):
    if m is not None:
        flatten(m).zero_grad()
losses[0].backward()
torch.cuda.synchronize()
params = tm.named_params(("encz", fm.encz_model), ("ed", fm.encdec_model))
g64 = tm.oracle_elbo_grads(kw, g, torch.float64, spec.get("multiplier", 1.0), spec.get("prior"))
rng = np.random.default_rng(1)
xs = [tm.t(g[k] * (1 + 1e-7 * rng.standard_normal(g[k].shape))) for k in ("xt", "x2t", "x3t")]
gp = tm.oracle_elbo_grads(kw, g, torch.float64, spec.get("multiplier", 1.0), spec.get("prior"),
                          xs=xs)
g32 = {n: tm.t(g["grad/" + n]) for n, _ in params if "grad/" + n in g.files}
rows = []
for n, p in params:
    if n not in g64:
        continue
    rows.append((n, rel(p.main_grad, g64[n]), rel(g32[n], g64[n]) if n in g32 else -1,
                 rel(gp[n], g64[n])))
rows.sort(key=lambda r: -r[1])
print(f"{'tensor':40s} {'hip':>10s} {'ref32':>10s} {'fp64 pert':>10s}")
for r in rows[:25]:
    print(f"{r[0][:40]:40s} {r[1]:10.3e} {r[2]:10.3e} {r[3]:10.3e}")
print("median", np.median([r[1] for r in rows]), np.median([r[2] for r in rows]),
      np.median([r[3] for r in rows]))
