"""Whole-step HIP graph (vae2.graph.StepGraph) == eager steps, bit for bit.

Two identically seeded models take the same steps on the same clips and noise:
one eagerly, one through warm-up steps + captured-graph replays.  Parameters,
Adam moments, BN running statistics and the losses must agree exactly (every
kernel is deterministic, so replay changes nothing but the launch path)."""
import pytest
import torch

from helpers import build, make_cfg

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(arch, B, hw, seed=0):
    from vae2.model import FullModel_encdec
    from vae2.optim import FusedAdam
    ed, ez = build(make_cfg(arch, hw=hw), seed=seed)
    fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(DEV)
    fm.train()
    fm.defer_checks = True
    opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-3)
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(B, 9, *hw, generator=g).to(DEV) for _ in range(3)]
    eps = torch.randn(B, ez.z_dim, 1, 1, generator=g).to(DEV)
    code = torch.randn(B, ez.z_dim, 1, 1, generator=g).to(DEV)

    def step():
        opt.zero_grad()
        fm.set_noise(eps, code)
        return fm(*xs, 1.0)[0][0]
    return fm, opt, step


def _full_step(fm, opt, fwd):
    def f():
        loss = fwd()
        loss.backward()
        opt.step()
        return loss
    return f


@pytest.mark.parametrize("arch,B,hw", [("tiny", 2, (32, 64)), ("w18", 2, (64, 128))])
def test_graph_replay_matches_eager(arch, B, hw):
    from vae2.graph import StepGraph
    fa, oa, sa = _setup(arch, B, hw)
    fb, ob, sb = _setup(arch, B, hw)
    step_a = _full_step(fa, oa, sa)
    step_b = _full_step(fb, ob, sb)
    losses_a = [float(step_a()) for _ in range(5)]
    g = StepGraph(step_b, warmup=2)  # executes 2 eager steps, captures the 3rd
    losses_b = []
    for _ in range(3):
        losses_b.append(float(g.replay()))
    torch.cuda.synchronize()
    assert losses_a[2:] == losses_b, (losses_a, losses_b)
    for fa_, fb_ in zip(oa.flats, ob.flats):
        assert torch.equal(fa_.data, fb_.data)
    for ma, mb in zip(oa.exp_avg + oa.exp_avg_sq, ob.exp_avg + ob.exp_avg_sq):
        assert torch.equal(ma, mb)
    assert oa.step_count == ob.step_count == 5
    ba = dict(fa.named_buffers())
    for name, buf in fb.named_buffers():
        assert torch.equal(buf, ba[name]), name
