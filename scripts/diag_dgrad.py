"""Diagnostic: discriminator weight gradients, HIP vs fp64 oracle, per call."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")]
import torch, numpy as np
from helpers import build, make_cfg, golden, t, rel
from oracle import ref_cpu
from vae2 import ops
from vae2.params import flatten
g = golden("tiny_gan")
x2t, x2p = t(g["x2t"]), t(g["x2p"])
for label, real in (("real", True), ("fake", False)):
    for which in ("ds", "df"):
        nets = build(make_cfg("tiny"), with_d=True)
        d = nets[2] if which == "ds" else nets[3]
        d64 = build(make_cfg("tiny"), with_d=True)[2 if which == "ds" else 3].double()
        x = x2t if real else x2p
        if which == "df":
            x = x[:, 3:6]
        out = ref_cpu.lsgan(ref_cpu.run_dsc(d64, x.double()), real) * 0.5 / 1
        out.backward()
        d = d.cuda()
        fl = flatten(d)
        fl.zero_grad()
        y = d.run(ops.to_nhwc(x.cuda().contiguous()))
        l = ops.lsgan(y, real, 0.5 / x.shape[0])
        l.backward()
        torch.cuda.synchronize()
        print(label, which, "loss", float(l), float(out))
        errs = []
        for (n, p), (_, q) in zip(d.named_parameters(), d64.named_parameters()):
            if q.grad is None or float(q.grad.norm()) == 0:
                continue
            errs.append((rel(p.main_grad, q.grad), n, float(q.grad.norm())))
        errs.sort(reverse=True)
        for e in errs[:6]:
            print("   %.3e %s |g|=%.3e" % e)
