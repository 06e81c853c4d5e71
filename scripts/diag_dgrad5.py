"""Diagnostic: full D (real, sequence) with the head loss; gradient at every stage boundary."""
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


def cpu(dt):
    d = build(make_cfg("tiny"), with_d=True)[2].to(dt)
    taps = []

    def tap(v, name):
        v.retain_grad()
        taps.append((name, v))
        return v
    xx = x.to(dt)
    h = tap(F.relu(ref_cpu._bn(ref_cpu._conv(xx, d.conv1), d.bn1)), "stem1")
    h = tap(F.relu(ref_cpu._bn(ref_cpu._conv(h, d.conv2), d.bn2)), "stem2")
    h = tap(ref_cpu._blocks(d.layer1, h), "layer1")
    ys = [h]
    for s in (2, 3):
        xs = ref_cpu._transition(getattr(d, f"transition{s-1}"), ys, getattr(d, f"stage{s}_cfg")["NUM_BRANCHES"])
        xs = [tap(v, f"t{s-1}_{i}") for i, v in enumerate(xs)]
        for m in getattr(d, f"stage{s}"):
            xs = ref_cpu._hr_module(m, xs)
        ys = [tap(v, f"s{s}_{i}") for i, v in enumerate(xs)]
    xs = ref_cpu._transition(d.transition3, ys, 4)
    xs = [tap(v, f"t3_{i}") for i, v in enumerate(xs)]
    ys = ref_cpu._stage4(d, "", xs)
    ys = [tap(v, f"s4_{i}") for i, v in enumerate(ys)]
    out = ref_cpu._seq(d.last_layer, ref_cpu._upcat(ys))
    ref_cpu.lsgan(out, True).backward()
    return {n: v.grad.double() for n, v in taps}, d


r64, d64 = cpu(torch.float64)
r32, d32 = cpu(torch.float32)
d = build(make_cfg("tiny"), with_d=True)[2].cuda()
flatten(d).zero_grad()
grads = {}


def tap(v, name):
    v.register_hook(lambda gr: grads.__setitem__(name, gr.detach().clone()))
    return v
h = ops.to_nhwc(x.cuda().contiguous())
h = tap(ops.conv_bn(h, d.conv1, d.bn1, relu=True), "stem1")
h = tap(ops.conv_bn(h, d.conv2, d.bn2, relu=True), "stem2")
h = tap(hrnet.run_seq(d.layer1, h), "layer1")
ys = [h]
for s in (2, 3):
    xs = hrnet.run_transition(getattr(d, f"transition{s-1}"), ys, getattr(d, f"stage{s}_cfg")["NUM_BRANCHES"])
    xs = [tap(v, f"t{s-1}_{i}") if v.requires_grad else v for i, v in enumerate(xs)]
    ys = hrnet.run_stage(getattr(d, f"stage{s}"), xs)
    ys = [tap(v, f"s{s}_{i}") for i, v in enumerate(ys)]
xs = hrnet.run_transition(d.transition3, ys, 4)
xs = [tap(v, f"t3_{i}") for i, v in enumerate(xs)]
ys = hrnet.run_stage(d.stage4, xs)
ys = [tap(v, f"s4_{i}") for i, v in enumerate(ys)]
from vae2 import heads as vheads
out = vheads.run([d.last_layer], ys)
ops.lsgan(out, True, 0.5).backward()
torch.cuda.synchronize()
for n in r64:
    if n in grads:
        hg = grads[n].permute(0, 3, 1, 2).double().cpu()
        print("%-8s hip %.3e cpu32 %.3e |g| %.3e" % (n, rel(hg, r64[n]), rel(r32[n], r64[n]), float(r64[n].norm())))
errs = sorted([(rel(p.main_grad, q.grad), n) for (n, p), (_, q) in zip(d.named_parameters(), d64.named_parameters()) if float(q.grad.norm()) > 1e-9], reverse=True)
print(errs[:5])
