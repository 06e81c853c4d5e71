"""Diagnostic: discriminator head alone (ys as leaves): fused vs generic, +/- final conv."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.nn.functional as F
from helpers import build, make_cfg, golden, t, rel
from oracle import ref_cpu
from vae2 import ops, hrnet
from vae2 import heads as vheads
from vae2.params import flatten
g = golden("tiny_gan")
x = t(g["x2t"])
d64 = build(make_cfg("tiny"), with_d=True)[2].double()
with torch.no_grad():
    ys64 = ref_cpu._stage4(d64, "", ref_cpu._trunk(d64, "", x.double()))
dh = build(make_cfg("tiny"), with_d=True)[2].cuda()
with torch.no_grad():
    ysh = hrnet.run_stage(dh.stage4, dh._trunk_to_stage4_inputs("", ops.to_nhwc(x.cuda().contiguous())))
nchw = lambda a: a.permute(0, 3, 1, 2).double().cpu()
for src in ("cpu64->f32", "hip"):
    for variant in ("fused+final", "generic+final", "generic_nofinal"):
        ys_ref = [y.clone().requires_grad_(True) for y in ys64]
        if variant == "generic_nofinal":
            out = F.relu(ref_cpu._seq(d64.last_layer[:2], ref_cpu._upcat(ys_ref)))
        else:
            out = ref_cpu._seq(d64.last_layer, ref_cpu._upcat(ys_ref))
        ((out - 1) ** 2).sum().backward()
        d = build(make_cfg("tiny"), with_d=True)[2].cuda()
        flatten(d).zero_grad()
        base = [ops.to_nhwc(y.float().cuda()) for y in ys64] if src.startswith("cpu") else ysh
        ys = [b.detach().clone().requires_grad_(True) for b in base]
        if variant == "fused+final":
            o = vheads.run([d.last_layer], ys)
        elif variant == "generic+final":
            o = hrnet.run_head(d.last_layer, ops.up_cat(ys))
        else:
            o = ops.conv_bn(ops.up_cat(ys), d.last_layer[0], d.last_layer[1], True)
        ops.lsgan(o, True, 1.0).backward()
        torch.cuda.synchronize()
        print(src, variant, "dY rel:", ["%.2e" % rel(nchw(a.grad), b.grad) for a, b in zip(ys, ys_ref)])
        for y in ys_ref:
            y.grad = None
# fp64 reference evaluated at HIP's ys
ys_h64 = [nchw(y).clone().requires_grad_(True) for y in ysh]
out = ref_cpu._seq(d64.last_layer, ref_cpu._upcat(ys_h64))
((out - 1) ** 2).sum().backward()
d = build(make_cfg("tiny"), with_d=True)[2].cuda()
flatten(d).zero_grad()
ys = [b.detach().clone().requires_grad_(True) for b in ysh]
ops.lsgan(vheads.run([d.last_layer], ys), True, 1.0).backward()
torch.cuda.synchronize()
print("fp64-at-hip-ys vs hip:", ["%.2e" % rel(nchw(a.grad), b.grad) for a, b in zip(ys, ys_h64)])
print("ys hip vs 64 per-branch rel:", ["%.2e" % rel(nchw(a), b) for a, b in zip(ysh, ys64)])
ys_c = [ops.to_nhwc(y.float().cuda()) for y in ys64]
print("ys cpu->f32 vs 64 per-branch rel:", ["%.2e" % rel(nchw(a), b) for a, b in zip(ys_c, ys64)])
u64 = ref_cpu._upcat(ys64)
r64 = ref_cpu._conv(u64, d64.last_layer[0])
rh = ref_cpu._conv(ref_cpu._upcat([nchw(y) for y in ysh]), d64.last_layer[0])
dr = rh - r64
print("r: std per ch", [round(float(r64[:, k].std()), 6) for k in range(0, 60, 12)],
      " |dr| per ch mean", [float(dr[:, k].mean()) for k in range(0, 60, 12)],
      " dr std", [float(dr[:, k].std()) for k in range(0, 60, 12)])
