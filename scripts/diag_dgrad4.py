"""Diagnostic: per-tensor gradients through the D trunk with the conv+BN head loss."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.nn.functional as F
from helpers import build, make_cfg, golden, t, rel
from oracle import ref_cpu
from vae2 import ops, hrnet
from vae2.params import flatten
g = golden("tiny_gan")
x = t(g["x2t"])
res = {}
for dt in (torch.float64, torch.float32):
    d = build(make_cfg("tiny"), with_d=True)[2].to(dt)
    xs = ref_cpu._trunk(d, "", x.to(dt))
    xs = [v.detach().requires_grad_(True) for v in xs]
    ys = ref_cpu._stage4(d, "", xs)
    for y in ys: y.retain_grad()
    u = ref_cpu._upcat(ys)
    u.retain_grad()
    h = F.relu(ref_cpu._bn(ref_cpu._conv(u, d.last_layer[0]), d.last_layer[1]))
    ((h - 1) ** 2).sum().backward()
    res[dt] = dict(xs=[v.detach() for v in xs], xg=[v.grad.double() for v in xs],
                   yg=[y.grad.double() for y in ys], ug=u.grad.double(), u=u.detach().double())
d = build(make_cfg("tiny"), with_d=True)[2].cuda()
flatten(d).zero_grad()
xs = [ops.to_nhwc(v.float().cuda()).detach().requires_grad_(True) for v in res[torch.float32]["xs"]]
ys = hrnet.run_stage(d.stage4, xs)
grads = {}
for i, y in enumerate(ys):
    y.register_hook(lambda gr, i=i: grads.__setitem__(("y", i), gr.detach().clone()))
u = ops.up_cat(ys)
u.register_hook(lambda gr: grads.__setitem__("u", gr.detach().clone()))
h = ops.conv_bn(u, d.last_layer[0], d.last_layer[1], True)
ops.lsgan(h, True, 1.0).backward()
torch.cuda.synchronize()
nchw = lambda a: a.permute(0, 3, 1, 2).double().cpu()
r64, r32 = res[torch.float64], res[torch.float32]
print("u fwd hip vs 64", rel(nchw(u), r64["u"]), "cpu32", rel(r32["u"], r64["u"]))
print("ug hip", rel(nchw(grads["u"]), r64["ug"]), "cpu32", rel(r32["ug"], r64["ug"]))
for i in range(4):
    print("yg", i, "hip", rel(nchw(grads[("y", i)]), r64["yg"][i]), "cpu32", rel(r32["yg"][i], r64["yg"][i]),
          "|g|", float(r64["yg"][i].norm()))
for i in range(4):
    print("xg", i, "hip", rel(nchw(xs[i].grad), r64["xg"][i]), "cpu32", rel(r32["xg"][i], r64["xg"][i]))
