"""Diagnostic: gradient at the head's input (upcat output) and BN stats, HIP vs fp64."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.nn.functional as F
from helpers import build, make_cfg, golden, t, rel, max_rel
from oracle import ref_cpu
from vae2 import ops, hrnet
from vae2.params import flatten
g = golden("tiny_gan")
x = t(g["x2t"])
res = {}
for dt in (torch.float64, torch.float32):
    d = build(make_cfg("tiny"), with_d=True)[2].to(dt)
    ys = ref_cpu._stage4(d, "", ref_cpu._trunk(d, "", x.to(dt)))
    u = ref_cpu._upcat(ys).detach().requires_grad_(True)
    r = ref_cpu._conv(u, d.last_layer[0])
    r.retain_grad()
    h = F.relu(ref_cpu._bn(r, d.last_layer[1]))
    loss = ((h - 1) ** 2).sum()
    loss.backward()
    res[dt] = dict(u=u.detach().double(), ug=u.grad.double(), r=r.detach().double(), rg=r.grad.double())
d = build(make_cfg("tiny"), with_d=True)[2].cuda()
flatten(d).zero_grad()
u = ops.to_nhwc(res[torch.float32]["u"].float().cuda()).detach().requires_grad_(True)
h = ops.conv_bn(u, d.last_layer[0], d.last_layer[1], True)
loss = ops.lsgan(h, True, 1.0)
loss.backward()
torch.cuda.synchronize()
ug = u.grad.permute(0, 3, 1, 2).double().cpu()
r64 = res[torch.float64]
print("u fp32 vs fp64", rel(res[torch.float32]["u"], r64["u"]))
print("ug cpu32 vs 64", rel(res[torch.float32]["ug"], r64["ug"]), " hip vs 64", rel(ug, r64["ug"]))
rr = r64["r"]
print("r mean/std per ch:", [(round(float(rr[:, c].mean()), 4), round(float(rr[:, c].std()), 5)) for c in range(0, 60, 10)])
print("rg cpu32 vs 64", rel(res[torch.float32]["rg"], r64["rg"]))
# per-channel error of ug
e = (ug - r64["ug"]).norm(dim=(0, 2, 3)) / r64["ug"].norm(dim=(0, 2, 3))
print("per-channel ug rel err (hip):", [round(float(v), 5) for v in e[:12]])
