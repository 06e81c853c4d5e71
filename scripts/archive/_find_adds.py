# Diagnostic: which ATen add kernels (autograd gradient accumulation) remain in one
# bench-geometry training step, with their shapes.   gpurun -- python scripts/_find_adds.py
import sys, os, collections
sys.path.insert(0, 'vae-2_amd'); sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import torch
from helpers import build, make_cfg
from vae2.model import FullModel_encdec
from vae2.optim import FusedAdam
dev = 'cuda'
ed, ez = build(make_cfg(arch='w18', hw=(128, 256)))
fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(dev)
opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-4)
xs = [torch.randn(8, 9, 128, 256, device=dev) for _ in range(3)]
def step():
    fm.set_noise(torch.randn(8, 10, 1, 1, device=dev), torch.randn(8, 10, 1, 1, device=dev))
    opt.zero_grad(); l = fm(*xs, 1.0)[0][0]; l.backward(); opt.step()
step(); torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=False) as p:
    step(); torch.cuda.synchronize()
cnt = collections.Counter()
for e in p.events():
    if e.name in ('aten::add', 'aten::add_') :
        cnt[(e.name, str(e.input_shapes)[:120])] += 1
for k, v in cnt.most_common(30): print(v, k)
