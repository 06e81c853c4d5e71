"""Flat parameter / gradient buffers.

All parameters of a module tree are re-pointed into one contiguous fp32 device
buffer, and each gets `main_grad`, a view into a matching flat gradient buffer
that the HIP backward kernels accumulate into.  One buffer per model means one
fused Adam launch per step and one RCCL all-reduce (or a few buckets) for data
parallelism instead of ~1,000 per-tensor operations.  Parameter objects keep
their identity and names, so state_dicts are unchanged.
"""
import torch


class FlatParams:
    def __init__(self, module, device=None):
        seen = set()
        self.params = []
        self.names = []
        for name, p in module.named_parameters():
            if id(p) in seen:
                continue
            seen.add(id(p))
            self.params.append(p)
            self.names.append(name)
        if not self.params:
            raise ValueError("module has no parameters")
        device = device or self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.numel = total
        self.data = torch.empty(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        self.offsets = []
        off = 0
        with torch.no_grad():
            for p in self.params:
                n = p.numel()
                self.data[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.data[off:off + n].view_as(p)
                p.main_grad = self.grad[off:off + n].view_as(p)
                p.grad = None
                self.offsets.append(off)
                off += n

    def zero_grad(self):
        self.grad.zero_()

    def expose_grads(self):
        """Point each parameter's .grad at its slice of the flat gradient."""
        for p in self.params:
            p.grad = p.main_grad


def flatten(module, device=None):
    """Attach (once) and return the FlatParams of `module`."""
    fp = getattr(module, "_vae2_flat", None)
    if fp is None:
        fp = FlatParams(module, device)
        object.__setattr__(module, "_vae2_flat", fp)
    return fp
