"""Diagnostic: bisect the discriminator gradient error (trunk vs head), HIP vs fp64."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")]
import torch
from helpers import build, make_cfg, golden, t, rel
from oracle import ref_cpu
from vae2 import ops, hrnet
from vae2.params import flatten
g = golden("tiny_gan")
x = t(g["x2t"])


def oracle(mode, dt):
    d = build(make_cfg("tiny"), with_d=True)[2].to(dt)
    ys = ref_cpu._stage4(d, "", ref_cpu._trunk(d, "", x.to(dt)))
    if mode == "trunk":
        loss = sum(((y - 1) ** 2).sum() for y in ys)
    elif mode == "upcat":
        loss = ((ref_cpu._upcat(ys) - 1) ** 2).sum()
    elif mode == "conv":
        loss = ((ref_cpu._conv(ref_cpu._upcat(ys), d.last_layer[0]) - 1) ** 2).sum()
    elif mode == "convbn":
        loss = ((ref_cpu._seq(d.last_layer[:3], ref_cpu._upcat(ys)) - 1) ** 2).sum()
    else:
        loss = ((ref_cpu._seq(d.last_layer, ref_cpu._upcat(ys)) - 1) ** 2).sum()
    loss.backward()
    return d, float(loss)


def hip(mode):
    d = build(make_cfg("tiny"), with_d=True)[2].cuda()
    fl = flatten(d)
    fl.zero_grad()
    xs = d._trunk_to_stage4_inputs("", ops.to_nhwc(x.cuda().contiguous()))
    ys = hrnet.run_stage(d.stage4, xs)
    if mode == "trunk":
        loss = ops.weighted_sum([ops.lsgan(y, True, 1.0) for y in ys], [1.0] * len(ys))
    elif mode == "upcat":
        loss = ops.lsgan(ops.up_cat(ys), True, 1.0)
    elif mode == "conv":
        loss = ops.lsgan(ops.conv(ops.up_cat(ys), d.last_layer[0]), True, 1.0)
    elif mode == "convbn":
        loss = ops.lsgan(ops.conv_bn(ops.up_cat(ys), d.last_layer[0], d.last_layer[1], True),
                         True, 1.0)
    else:
        loss = ops.lsgan(d.run(ops.to_nhwc(x.cuda().contiguous())), True, 1.0) if mode == "full" \
            else ops.lsgan(hrnet.run_head(d.last_layer, ops.up_cat(ys)), True, 1.0)
    loss.backward()
    torch.cuda.synchronize()
    return d, float(loss)


for mode in ("conv", "convbn", "full"):
    d64, l64 = oracle("full" if mode == "head_generic" else mode, torch.float64)
    d32, l32 = oracle("full" if mode == "head_generic" else mode, torch.float32)
    dh, lh = hip(mode)
    errs = []
    for (n, p), (_, q), (_, r) in zip(dh.named_parameters(), d64.named_parameters(),
                                      d32.named_parameters()):
        if q.grad is None or float(q.grad.norm()) < 1e-9:
            continue
        errs.append((rel(p.main_grad, q.grad), rel(r.grad, q.grad), n))
    errs.sort(reverse=True)
    print(mode, "loss hip %.8g fp64 %.8g" % (lh, l64))
    for e in errs[:4]:
        print("   hip %.3e  cpu32 %.3e  %s" % e)
