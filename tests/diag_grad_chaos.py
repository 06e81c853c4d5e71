"""How chaotic is the ELBO gradient of HRNet-W18 in its inputs? (test infrastructure: CPU
oracle only; not collected by pytest)

Config 2 geometry (64x64, L=2, 2 classes, B=4), the Kaiming-scale state of
tests/test_bf16_gpu.py::_kaiming_grads (same seeds).  Runs oracle/ref_cpu.elbo in fp64,
then again with the three clips scaled by (1 + e * N(0,1)) for several e, and prints the
per-tensor gradient cosine to the unperturbed fp64 gradient (min / p10 / median), the fp32
oracle's cosine, and the tensors whose cosine stays above 0.99 at e = 2e-3 (about a bf16
rounding): those are test_bf16_gpu.STABLE.

    python tests/diag_grad_chaos.py        # ~2 minutes on 8 cores

Round 4 output (tests/test_bf16_gpu.py docstring): fp32 median 0.998 (min 0.991);
e = 1e-7 median 0.9995, 1e-5 0.945, 1e-4 0.50, 2e-3 0.013; 16 stable tensors, all in the
decoders' output heads.
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "vae-2_amd")]

from helpers import build, make_cfg  # noqa: E402
from oracle import ref_cpu  # noqa: E402
from test_model_gpu import named_params  # noqa: E402

KW = dict(arch="w18", hw=(64, 64), L=2, classes=2)


def inputs():
    # the draw order of test_bf16_gpu._inputs(seed=17)
    gen = torch.Generator().manual_seed(17)
    xs = [torch.randn(4, 6, 64, 64, generator=gen) for _ in range(3)]
    eps = torch.randn(4, 10, 1, 1, generator=gen)
    code = torch.randn(4, 10, 1, 1, generator=gen)
    return xs, eps, code


def grads(dtype, e=0.0):
    xs, eps, code = inputs()
    torch.manual_seed(0)
    ed, ez = build(make_cfg(**KW))
    ed, ez = ed.to(dtype), ez.to(dtype)
    params = named_params(("encz", ez), ("ed", ed))
    gen = torch.Generator().manual_seed(21)
    with torch.no_grad():
        for _, p in params:
            if p.dim() >= 2:
                std = (2.0 / p[0].numel()) ** 0.5
                p.copy_((torch.randn(p.shape, generator=gen) * std).to(dtype))
    xs = [x.to(dtype) for x in xs]
    if e:
        pg = torch.Generator().manual_seed(77)
        xs = [x * (1 + e * torch.randn(x.shape, generator=pg, dtype=dtype)) for x in xs]
    terms, _, _ = ref_cpu.elbo(ez, ed, *xs, eps.to(dtype), code.to(dtype))
    terms["loss_all"].backward()
    return {n: p.grad.detach().double() for n, p in params if p.grad is not None}


def cosines(a, b):
    big = max(float(v.norm()) for v in a.values())
    return {n: float((a[n] * b[n]).sum() / (a[n].norm() * b[n].norm() + 1e-300))
            for n in a if float(a[n].norm()) > 1e-4 * big}


def report(tag, c):
    v = sorted(c.values())
    print(f"{tag}: {len(v)} tensors, min {v[0]:.4f} p10 {v[len(v) // 10]:.4f} "
          f"median {v[len(v) // 2]:.4f}")


if __name__ == "__main__":
    g64 = grads(torch.float64)
    report("fp32 oracle", cosines(g64, grads(torch.float32)))
    for e in (1e-7, 1e-5, 1e-4, 2e-3):
        c = cosines(g64, grads(torch.float64, e))
        report(f"fp64, inputs perturbed {e:g}", c)
    print("stable at 2e-3:", sorted(n for n, v in c.items() if v > 0.99))
