"""Adam over flat parameter buffers (torch.optim.Adam semantics, train.py:251-261).

One vae2_adam_step_dev launch per flat buffer; the math follows torch.optim.Adam
(lerp first moment, L2 weight decay folded into the gradient, bias corrections
in double).  The step counter and learning rate live in device memory
(vae2_adam_coeffs advances them), so the whole step can be captured in a HIP
graph and replayed (vae2.graph.StepGraph); change the learning rate through
param_groups[0]["lr"] and the next eager step() — or set_lr() between replays.  state_dict() / load_state_dict() use torch.optim.Adam's format
(per-parameter exp_avg / exp_avg_sq / step) so optimizer checkpoints interchange.
"""

import torch

from . import ops, streams
from ._lib import call
from .params import flatten


class FusedAdam:
    def __init__(self, modules, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if not isinstance(modules, (list, tuple)):
            modules = [modules]
        self.flats = [flatten(m) for m in modules]
        # packed conv weights, refreshed in one launch per model after every update
        self.packs = [ops.PackPlan(m) for m in modules]
        self.lr = float(lr)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        dev = self.flats[0].data.device
        self._state = torch.zeros(2, dtype=torch.float64, device=dev)  # {step, lr}
        self._coeffs = torch.zeros(2, dtype=torch.float32, device=dev)
        self._dev_lr = None
        self.exp_avg = [torch.zeros_like(f.data) for f in self.flats]
        self.exp_avg_sq = [torch.zeros_like(f.data) for f in self.flats]
        self.param_groups = [{"params": [p for f in self.flats for p in f.params], "lr": self.lr,
                              "betas": self.betas, "eps": self.eps,
                              "weight_decay": self.weight_decay, "amsgrad": False,
                              "maximize": False, "foreach": None, "capturable": False,
                              "differentiable": False, "fused": None}]

    def zero_grad(self, set_to_none=False):
        streams.join_all()
        for f in self.flats:
            f.zero_grad()

    @property
    def step_count(self):
        return int(self._state[0].item())

    @step_count.setter
    def step_count(self, n):
        self._state[0].fill_(float(n))

    def set_lr(self, lr):
        self.param_groups[0]["lr"] = float(lr)
        self._sync_lr()

    def _sync_lr(self):
        lr = float(self.param_groups[0]["lr"])
        self.lr = lr
        if lr != self._dev_lr:  # eager: graphs read the device copy on replay
            self._state[1].fill_(lr)
            self._dev_lr = lr

    @torch.no_grad()
    def step(self):
        self._sync_lr()
        streams.join_all()
        s = ops.stream_ptr()
        call("vae2_adam_coeffs", ops.ptr(self._state), self.betas[0], self.betas[1],
             ops.ptr(self._coeffs), s)
        for f, m, v in zip(self.flats, self.exp_avg, self.exp_avg_sq):
            call("vae2_adam_step_dev", ops.ptr(f.data), ops.ptr(f.grad), ops.ptr(m), ops.ptr(v),
                 f.numel, ops.ptr(self._coeffs), self.betas[0], self.betas[1], self.eps,
                 self.weight_decay, s)
        for plan in self.packs:
            plan.bump_versions()

    # ---- torch.optim.Adam-compatible checkpoint format ----
    def state_dict(self):
        state = {}
        idx = 0
        step = float(self.step_count)
        for f, m, v in zip(self.flats, self.exp_avg, self.exp_avg_sq):
            for p, off in zip(f.params, f.offsets):
                n = p.numel()
                state[idx] = {"step": torch.tensor(step),
                              "exp_avg": m[off:off + n].view_as(p).clone(),
                              "exp_avg_sq": v[off:off + n].view_as(p).clone()}
                idx += 1
        group = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        group["params"] = list(range(idx))
        return {"state": state, "param_groups": [group]}

    @torch.no_grad()
    def load_state_dict(self, sd):
        st = sd["state"]
        idx = 0
        steps = []
        for f, m, v in zip(self.flats, self.exp_avg, self.exp_avg_sq):
            for p, off in zip(f.params, f.offsets):
                n = p.numel()
                if idx in st:
                    m[off:off + n].copy_(st[idx]["exp_avg"].reshape(-1))
                    v[off:off + n].copy_(st[idx]["exp_avg_sq"].reshape(-1))
                    steps.append(int(float(st[idx]["step"])))
                idx += 1
        if steps:
            self.step_count = max(steps)
        g = sd["param_groups"][0]
        self.param_groups[0]["lr"] = g.get("lr", self.lr)
        self._sync_lr()
        self.betas = tuple(g.get("betas", self.betas))
        self.eps = g.get("eps", self.eps)
        self.weight_decay = g.get("weight_decay", self.weight_decay)

