"""Diagnostic (GPU): BasicBlock / fuse backward accuracy vs fp64 at the stage-4 branch
shapes, B=8, with the fp32 CPU distance and the fp64 1e-6-perturbation sensitivity.
    python scripts/diag_block.py"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vae-2_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from helpers import build, make_cfg, rel  # noqa: E402
from oracle import ref_cpu  # noqa: E402

DEV = "cuda"
B, H, W = 8, 128, 256


def nchw(v):
    return v.permute(0, 3, 1, 2).detach().cpu()


def run_block(blk, x, gout, algo=0, batched=True):
    from vae2 import _lib, hrnet, ops
    lib = _lib.load()
    prev = lib.vae2_conv2d_set_algo(algo)
    ops.BN_BATCH = batched
    try:
        bg = copy.deepcopy(blk).to(DEV)
        xg = ops.new_act((x.shape[0], x.shape[2], x.shape[3], x.shape[1]), torch.empty(1, device=DEV))
        with torch.no_grad():
            xg.copy_(x.permute(0, 2, 3, 1).to(DEV))
        xg.requires_grad_()
        y = hrnet.run_blocks_lockstep([bg], [xg])[0]
        y.backward(gout.permute(0, 2, 3, 1).contiguous().to(DEV))
        torch.cuda.synchronize()
    finally:
        lib.vae2_conv2d_set_algo(prev)
        ops.BN_BATCH = True
    return bg, xg


def main():
    ed, _ = build(make_cfg(arch="w18", hw=(H, W)))
    mod = ed.stage4[0]
    g = torch.Generator().manual_seed(12)
    with torch.no_grad():
        for p in mod.modules():
            if isinstance(p, torch.nn.Conv2d):
                p.weight.normal_(0, (1.0 / p.weight[0].numel()) ** 0.5, generator=g)
            elif isinstance(p, torch.nn.BatchNorm2d):
                p.weight.uniform_(0.5, 1.5, generator=g)
                p.bias.normal_(0, 0.1, generator=g)
    shapes = [(18, H, W), (36, H // 2, W // 2), (72, H // 4, W // 4), (144, H // 8, W // 8)]
    for bi, (c, h, w) in enumerate(shapes):
        blk = mod.branches[bi][0]
        x = torch.randn(B, c, h, w, generator=g)
        gout = torch.randn(B, c, h, w, generator=g)
        res = {}
        for tag, dt, pert in (("f64", torch.float64, 0), ("f32", torch.float32, 0),
                              ("f64p", torch.float64, 1e-6)):
            m = copy.deepcopy(blk).to(dt)
            xx = x.detach().clone().to(dt)
            if pert:
                xx = xx * (1 + pert * torch.randn(x.shape, generator=g, dtype=dt))
            xx = xx.detach().requires_grad_()
            y = ref_cpu._block(m, xx)
            y.backward(gout.to(dt))
            res[tag] = (m, xx)
        for algo in (0, 1, 2):
            for batched in (True, False):
                bg, xg = run_block(blk, x, gout, algo, batched)
                line = [f"x {rel(nchw(xg.grad), res['f64'][1].grad):.2e}"]
                for (n, p), (_, p64) in zip(bg.named_parameters(), res["f64"][0].named_parameters()):
                    line.append(f"{n} {rel(p.grad, p64.grad):.2e}")
                print(f"branch {bi} algo {algo} batched {batched}:", " ".join(line), flush=True)
        ref = [f"x {rel(res['f32'][1].grad, res['f64'][1].grad):.2e}/{rel(res['f64p'][1].grad, res['f64'][1].grad):.2e}"]
        for (n, p), (_, p64), (_, pp) in zip(res["f32"][0].named_parameters(),
                                             res["f64"][0].named_parameters(),
                                             res["f64p"][0].named_parameters()):
            ref.append(f"{n} {rel(p.grad, p64.grad):.2e}/{rel(pp.grad, p64.grad):.2e}")
        print(f"branch {bi} cpu32/sens:", " ".join(ref), flush=True)


if __name__ == "__main__":
    main()
