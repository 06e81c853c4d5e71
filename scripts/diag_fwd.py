"""Diagnostic: forward activations of the D trunk, HIP vs fp64, per stage / channel."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.nn.functional as F
from helpers import build, make_cfg, golden, t, rel, max_rel
from oracle import ref_cpu
from vae2 import ops, hrnet
g = golden("tiny_gan")
x = t(g["x2t"])
d64 = build(make_cfg("tiny"), with_d=True)[2].double()
d = build(make_cfg("tiny"), with_d=True)[2].cuda()
nchw = lambda a: a.permute(0, 3, 1, 2).double().cpu()
with torch.no_grad():
    c = ref_cpu._conv(x.double(), d64.conv1)
    hc = ops.conv(ops.to_nhwc(x.cuda().contiguous()), d.conv1)
    print("conv1 out rel", rel(nchw(hc), c), "max_rel", max_rel(nchw(hc), c))
    print("conv1 per-ch mean/std", [(round(float(c[:, k].mean()), 6), round(float(c[:, k].std()), 6)) for k in range(0, 64, 16)])
    a = F.relu(ref_cpu._bn(c, d64.bn1))
    ha = ops.conv_bn(ops.to_nhwc(x.cuda().contiguous()), d.conv1, d.bn1, relu=True)
    e = (nchw(ha) - a).abs().amax(dim=(0, 2, 3)) / a.abs().amax(dim=(0, 2, 3))
    print("stem1 out max-rel per channel top:", sorted([round(float(v), 7) for v in e], reverse=True)[:5])
    xs64 = ref_cpu._trunk(d64, "", x.double())
    ys64 = ref_cpu._stage4(d64, "", xs64)
    xs = d._trunk_to_stage4_inputs("", ops.to_nhwc(x.cuda().contiguous()))
    ys = hrnet.run_stage(d.stage4, xs)
    for i in range(4):
        print("t3", i, "max_rel", max_rel(nchw(xs[i]), xs64[i]), " s4", i, "max_rel", max_rel(nchw(ys[i]), ys64[i]))
