"""Parity of the HIP ELBO step with the reference (golden vectors) and the oracle.

Tolerances: the ELBO terms within 1e-5 relative (1e-4,
the north-star bar, for the HD_Z KL whose exp(lv) - lv - 1 cancels in fp32 at
lv ~ 1e-3); each network fed the reference's own inputs within 1e-4 relative
(x2t_hat, mu|logvar, each decoder on the golden x2t_hat); end-to-end decoder
frames within the reference's own fp32 spread (1e-3).  End-to-end gradients are
chaotic in fp32 (the reference's own fp32 gradients sit a median 1.1 % and up to
13 % from fp64 on the tiny net), so they are held to an fp64 oracle: per tensor
the HIP gradient must be no further from fp64 than the fp32 reference is (x3 of
its own distance or of the median distance, +1e-4), and the median distance
within 1.5x of the reference's.
"""
import copy

import numpy as np
import pytest
import torch

from helpers import build, golden, load_eval_state, make_cfg, max_rel, ref_checkpoint, rel, t

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = {
    "tiny_native": dict(arch="tiny"),
    "tiny_hdz": dict(arch="tiny", hd=True, z=3),
    "tiny_base": dict(arch="tiny", baseline=True),
    "w18": dict(arch="w18"),
}


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous().to(DEV)


def nchw(x):
    return x.permute(0, 3, 1, 2).detach().cpu()


def hip_model(kw, with_d=False, gan_lambda=0.0):
    """FullModel_encdec on the GPU with flat parameter / gradient buffers (main_grad)."""
    from vae2.model import FullModel_encdec
    from vae2.params import flatten
    nets = build(make_cfg(**kw), with_d=with_d)
    ed, ez = nets[:2]
    ds, df = nets[2:] if with_d else (None, None)
    fm = FullModel_encdec(ez, ed, ds, df, None, None, None, 1.0, 0.1, 1.0, gan_lambda).to(DEV)
    fm.train()
    for m in nets:
        if m is not None:
            flatten(m).zero_grad()
    return fm


def named_params(*pairs):
    out = []
    for prefix, m in pairs:
        if m is not None:
            out += list(m.named_parameters(prefix=prefix))
    return out


def oracle_elbo_grads(kw, g, dtype, multiplier=1.0, prior=False, with_d=False, gan_lambda=0.0,
                      xs=None, noise_=None, d_step=False, perturb=0.0, pseed=0):
    """Oracle ELBO (+ D step) gradients in `dtype` on golden (or given) inputs:
    {name: grad} with encz./ed. (and ds./df. for the D step) prefixes.  The D step's real
    sample is x2t, or x3t in baseline mode (function.py:503-504)."""
    from oracle import ref_cpu
    nets = build(make_cfg(**kw), with_d=with_d)
    nets = [n.to(dtype) if n is not None else None for n in nets]
    ed, ez = nets[:2]
    ds, df = nets[2:] if with_d else (None, None)
    if xs is None:
        xs = [t(g[k]) for k in ("xt", "x2t", "x3t")]
    xs = [x.to(dtype) for x in xs]
    if perturb:  # the reference's sensitivity to rounding-level input noise
        pg = torch.Generator().manual_seed(77 + pseed)
        xs = [x * (1 + perturb * torch.randn(x.shape, generator=pg, dtype=dtype)) for x in xs]
    det = kw.get("mode") == "DETERMINISTIC"
    if noise_ is None:
        noise_ = (None, None) if det else (t(g["eps"]), t(g["code"]))
    eps, code = (n.to(dtype) if n is not None else None for n in noise_)
    terms, preds, _ = ref_cpu.elbo(ez, ed, *xs, eps, code, multiplier=multiplier,
                                   is_baseline=kw.get("baseline", False),
                                   baseline_mode=kw.get("mode", "VAE_NATIVE"), prior=prior,
                                   ds=ds, df=df, gan_lambda=gan_lambda)
    terms["loss_all"].backward()
    grads = {n: p.grad.detach().float() for n, p in named_params(("encz", ez), ("ed", ed))
             if p.grad is not None}
    if d_step:
        for _, p in named_params(("ds", ds), ("df", df)):
            p.grad = None
        dl = ref_cpu.d_losses(ds, df, xs[2] if kw.get("baseline") else xs[1], preds[1])
        dl[0].backward()
        grads.update({n: p.grad.detach().float() for n, p in named_params(("ds", ds), ("df", df))})
    return grads


def check_grads_calibrated(params, g32, g64, ref_norms=None, floor=0.0, g64p=None):
    """Per tensor the HIP gradient must be no further from fp64 than the fp32
    reference is (x3 of its own distance or of the median distance, +1e-4), and the
    median distance within 1.5x of the reference's (fp32 gradients of
    this net are chaotic).  Analytically-zero tensors (conv biases in front of a
    BatchNorm) must stay ~0, and parameters the reference computes no gradient for
    (baseline decoders under no_grad) must get none.  ref_norms: the reference's fp32
    gradient norms (golden).  g64p: fp64 oracle gradients at inputs carrying 1e-6
    relative noise (one dict or several draws: the largest distance counts) — a tensor's
    distance between the two is the reference's own sensitivity to rounding-level input
    noise (ReLU masks an fp32 rounding flips) and widens that tensor's band like its fp32
    distance does."""
    for n, p in params:
        if n not in g64:
            assert float(p.main_grad.abs().max()) == 0.0, n
    if ref_norms is not None:
        ref_norms = [r for (n, _), r in zip(params, ref_norms) if n in g64]
    params = [(n, p) for n, p in params if n in g64]
    norms64 = np.array([float(g64[n].norm()) for n, _ in params])
    top = float(norms64.max())
    d_hip, d_ref, names = [], [], []
    for (n, p), n64 in zip(params, norms64):
        got = p.main_grad
        if n64 > 1e-6 * top:
            d_hip.append(rel(got, g64[n]))
            d_ref.append(rel(g32[n], g64[n]))
            names.append(n)
        else:
            assert float(got.norm()) <= 1e-3 * top, n
    med_ref = max(float(np.median(d_ref)), floor)
    if isinstance(g64p, dict):
        g64p = [g64p]
    sens = {n: max(rel(d[n], g64[n]) for d in g64p) for n in names} if g64p else {}
    for n, a, b in zip(names, d_hip, d_ref):
        assert a <= 3 * max(b, med_ref, sens.get(n, 0.0)) + 1e-4, (n, a, b, med_ref,
                                                                   sens.get(n))
    # the median band widens by the reference's median sensitivity the same way
    med_band = max(med_ref, float(np.median([sens[n] for n in names]))) if sens else med_ref
    assert np.median(d_hip) <= 1.5 * med_band + 1e-6, (np.median(d_hip), med_ref, med_band)
    if ref_norms is not None:  # |norm_hip - norm_ref32| within the same calibrated band
        for (n, p), rn, n64 in zip(params, ref_norms, norms64):
            if n64 > 1e-6 * top:
                dev = abs(float(p.main_grad.norm()) - rn) / n64
                ref_dev = abs(float(g32[n].norm()) - n64) / n64
                band = max(ref_dev, med_ref, sens.get(n, 0.0) if g64p else 0.0)
                assert dev <= 3 * band + 1e-4, (n, dev, ref_dev, med_ref, band)
    return float(np.median(d_hip)), med_ref


def oracle_grads(g, dtype):
    """Parameter gradients of the oracle ELBO step in `dtype` on the golden case."""
    from oracle import ref_cpu
    ed, ez = build(make_cfg("tiny"))
    ed, ez = ed.to(dtype), ez.to(dtype)
    xs = [t(g[k]).to(dtype) for k in ("xt", "x2t", "x3t")]
    terms, _, _ = ref_cpu.elbo(ez, ed, *xs, t(g["eps"]).to(dtype), t(g["code"]).to(dtype))
    terms["loss_all"].backward()
    return {n: p.grad.detach().float() for n, p in
            list(ez.named_parameters(prefix="encz")) + list(ed.named_parameters(prefix="ed"))}


def oracle_adam(g, dtype):
    """fp64 oracle version of the golden 3-step Adam run: (losses of steps 2-3,
    per-parameter sums after step 3, sorted by name)."""
    from oracle import ref_cpu
    ed, ez = build(make_cfg("tiny"))
    ed, ez = ed.to(dtype), ez.to(dtype)
    xs = [t(g[k]).to(dtype) for k in ("xt", "x2t", "x3t")]
    params = list(ez.named_parameters(prefix="encz")) + list(ed.named_parameters(prefix="ed"))
    opt = torch.optim.Adam([p for _, p in params], lr=1e-4)
    terms, _, _ = ref_cpu.elbo(ez, ed, *xs, t(g["eps"]).to(dtype), t(g["code"]).to(dtype))
    terms["loss_all"].backward()
    opt.step()
    traj = []
    for k in range(1, 3):
        opt.zero_grad()
        torch.manual_seed(200 + k)
        e, c = torch.randn(2, 4, 1, 1).to(dtype), torch.randn(2, 4, 1, 1).to(dtype)
        terms, _, _ = ref_cpu.elbo(ez, ed, *xs, e, c)
        traj.append(float(terms["loss_all"]))
        terms["loss_all"].backward()
        opt.step()
    psum = np.array([float(p.detach().double().sum()) for _, p in sorted(params)])
    return np.array(traj), psum


def noise(g, hd):
    eps = [t(g[f"eps{i}"]) for i in range(4)] if hd else t(g["eps"])
    return eps, t(g["code"])


@pytest.mark.parametrize("case", list(CASES))
def test_elbo_step_matches_reference(case):
    kw = CASES[case]
    g = golden(case)
    fm = hip_model(kw)
    fm.set_noise(*noise(g, kw.get("hd", False)))
    losses, x1p, x2p, x3p = fm(t(g["xt"]).to(DEV), t(g["x2t"]).to(DEV), t(g["x3t"]).to(DEV), 1.0,
                               is_baseline=kw.get("baseline", False))
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL"]
    for n, v in zip(names, losses[:5]):
        ref = float(g["loss_" + n])
        got = float(v.reshape(-1)[0]) if torch.is_tensor(v) else float(v)
        tol = 1e-4 if (n == "z_KL" and kw.get("hd", False)) else 1e-5
        assert abs(got - ref) <= tol * abs(ref) + 1e-7, (n, got, ref)
    assert max_rel(x2p, t(g["x2p"])) < 1e-4
    assert rel(x3p, t(g["x3p"])) < 1e-3
    assert rel(x1p, t(g["x1p"])) < 1e-3


@pytest.mark.parametrize("case", ["tiny_native", "w18"])
def test_each_network_on_golden_inputs(case):
    """Per-network parity (1e-4): each net is fed the reference's own inputs."""
    kw = CASES[case]
    g = golden(case)
    fm = hip_model(kw)
    ed, ez = fm.encdec_model, fm.encz_model
    with torch.no_grad():
        mv = ez.run(nhwc(torch.cat([t(g["xt"]), t(g["x3t"])], 1)))
        assert max_rel(nchw(mv), t(g["muvar"])) < 1e-4
        z = nhwc(t(g["z"]))
        x2p = ed.encode(nhwc(t(g["xt"])), z, nhwc(t(g["code"])))
        assert max_rel(nchw(x2p), t(g["x2p"])) < 1e-4
        gx2 = nhwc(t(g["x2p"]))
        x3p = ed.decode("decf_", gx2, z)
        x1p = ed.decode("decp_", gx2, z)
        assert max_rel(nchw(x3p), t(g["x3p"])) < 1e-4
        assert max_rel(nchw(x1p), t(g["x1p"])) < 1e-4


def test_grads_running_stats_and_adam_match_reference():
    from vae2.optim import FusedAdam
    g = golden("tiny_native")
    fm = hip_model(CASES["tiny_native"])
    ed, ez = fm.encdec_model, fm.encz_model
    opt = FusedAdam([ez, ed], lr=1e-4)
    xt, x2t, x3t = (t(g[k]).to(DEV) for k in ("xt", "x2t", "x3t"))
    fm.set_noise(*noise(g, False))
    opt.zero_grad()
    losses = fm(xt, x2t, x3t, 1.0)[0]
    losses[0].backward()
    params = list(ez.named_parameters(prefix="encz")) + list(ed.named_parameters(prefix="ed"))
    ref_norms = g["grad_norms"]
    floor = 1e-6 * ref_norms.max()
    g64 = oracle_grads(g, torch.float64)
    g32 = {n: t(g["grad/" + n]) for n, _ in params}  # the reference's own fp32 gradients
    d_hip, d_ref, names = [], [], []
    for (n, p), rn in zip(params, ref_norms):
        if rn > floor:
            d_hip.append(rel(p.main_grad, g64[n]))
            d_ref.append(rel(g32[n], g64[n]))
            names.append(n)
        else:  # analytically zero (conv bias in front of a BatchNorm)
            assert float(p.main_grad.norm()) <= 1e-3 * float(ref_norms.max()), n
    # Per tensor: no further from fp64 than 3x the reference's fp32 spread — its own,
    # or its median where the reference happened to land unusually close (a single
    # fp32 draw is as random as ours).  Overall: median within 1.5x of the reference's.
    med_ref = float(np.median(d_ref))
    for n, a, b in zip(names, d_hip, d_ref):
        assert a <= 3 * max(b, med_ref) + 1e-4, (n, a, b, med_ref)
    assert np.median(d_hip) <= 1.5 * med_ref, (np.median(d_hip), med_ref)
    # running statistics after the step
    rs = {("encz." + k): v for k, v in ez.state_dict().items() if "running" in k}
    rs.update({("ed." + k): v for k, v in ed.state_dict().items() if "running" in k})
    names = sorted(rs)
    assert names == list(g["running_names"])
    rsum = np.array([float(rs[k].double().sum()) for k in names])
    np.testing.assert_allclose(rsum, g["running_sum"], rtol=1e-4, atol=1e-6)
    # 3 Adam steps (lr 1e-4): Adam's normalised update amplifies the fp32 gradient
    # spread, so the trajectory is held to an fp64 oracle run: the HIP path must be
    # no further from it than the reference's own fp32 trajectory (x3, + 1e-6 rel).
    opt.step()
    traj = []
    for k in range(1, 3):
        opt.zero_grad()
        torch.manual_seed(200 + k)
        fm.set_noise(torch.randn(2, 4, 1, 1), torch.randn(2, 4, 1, 1))
        ls = fm(xt, x2t, x3t, 1.0)[0]
        traj.append(float(ls[0]))
        ls[0].backward()
        opt.step()
    t64, p64 = oracle_adam(g, torch.float64)
    d_ref = np.abs(np.asarray(g["adam_losses"]) - t64)
    d_hip = np.abs(np.asarray(traj) - t64)
    assert np.all(d_hip <= 3 * d_ref + 1e-6 * np.abs(t64)), (traj, list(g["adam_losses"]), t64)
    psum = np.array([float(p.detach().double().sum()) for _, p in sorted(params)])
    d_ref = np.abs(g["adam_param_sum"] - p64)
    d_hip = np.abs(psum - p64)
    assert np.median(d_hip) <= 3 * np.median(d_ref) + 1e-9


@pytest.mark.parametrize("L,hw,B", [(2, (64, 64), 4), (3, (36, 20), 2), (3, (128, 256), 2),
                                    (3, (256, 512), 2)])
def test_hip_matches_oracle_other_shapes(L, hw, B):
    """Config ② geometry (64x64, 2 ctx + 4 pred -> L=2, B=4), a ragged size, and the
    full-size geometries of configs ③/④ (128x256, the bench's) and ⑤ (256x512) at B=2
    so the CPU oracle finishes in seconds.  ELBO 1e-5 relative, x2t_hat 1e-4 max-rel,
    the decoder frames 1e-3 (the reference's own fp32 spread)."""
    from oracle import ref_cpu
    kw = dict(arch="w18", L=L, hw=hw, classes=L)  # 3 segments of L frames
    cfg = make_cfg(**kw)
    ed, ez = build(cfg)
    ed_c, ez_c = copy.deepcopy(ed), copy.deepcopy(ez)
    gen = torch.Generator().manual_seed(1)
    xs = [torch.randn(B, 3 * L, *hw, generator=gen) for _ in range(3)]
    eps = torch.randn(B, 10, 1, 1, generator=gen)
    code = torch.randn(B, 10, 1, 1, generator=gen)
    terms, preds, _ = ref_cpu.elbo(ez_c, ed_c, *xs, eps, code)
    from vae2.model import FullModel_encdec
    fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(DEV)
    fm.set_noise(eps, code)
    losses, x1p, x2p, x3p = fm(*[x.to(DEV) for x in xs], 1.0)
    ref = float(terms["loss_all"])
    assert abs(float(losses[0]) - ref) <= 1e-5 * abs(ref)
    assert max_rel(x2p, preds[1]) < 1e-4
    assert max_rel(x1p, preds[0]) < 1e-3
    assert max_rel(x3p, preds[2]) < 1e-3


MODE_CASES = {
    "tiny_anneal": dict(kw=dict(arch="tiny", mode="VAE_ANNEAL"), multiplier=0.37),
    "tiny_det": dict(kw=dict(arch="tiny", baseline=True, mode="DETERMINISTIC")),
    "tiny_prior": dict(kw=dict(arch="tiny"), prior=True),
}


@pytest.mark.parametrize("case", list(MODE_CASES))
def test_elbo_modes_match_reference(case):
    """VAE_ANNEAL (KL x multiplier), DETERMINISTIC (baseline, no posterior net, no code
    maps) and prior sampling: loss terms, x2t_hat and every gradient."""
    spec = MODE_CASES[case]
    kw = spec["kw"]
    g = golden(case)
    fm = hip_model(kw)
    det = kw.get("mode") == "DETERMINISTIC"
    if not det:
        fm.set_noise(t(g["eps"]), t(g["code"]))
    losses, x1p, x2p, x3p = fm(t(g["xt"]).to(DEV), t(g["x2t"]).to(DEV), t(g["x3t"]).to(DEV),
                               spec.get("multiplier", 1.0), is_baseline=kw.get("baseline", False),
                               baseline_mode=kw.get("mode", "VAE_NATIVE"),
                               sampling_mode="prior_sampling" if spec.get("prior") else "default")
    for n, v in zip(["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL"], losses[:5]):
        ref = float(g["loss_" + n])
        got = float(v.reshape(-1)[0]) if torch.is_tensor(v) else float(v)
        assert abs(got - ref) <= 1e-5 * abs(ref) + 1e-7, (n, got, ref)
    assert max_rel(x2p, t(g["x2p"])) < 1e-4
    from vae2.params import flatten
    for m in (fm.encz_model, fm.encdec_model):
        if m is not None:
            flatten(m).zero_grad()
    losses[0].backward()
    torch.cuda.synchronize()
    params = named_params(("encz", fm.encz_model), ("ed", fm.encdec_model))
    g64 = oracle_elbo_grads(kw, g, torch.float64, spec.get("multiplier", 1.0), spec.get("prior"))
    g32 = {n: t(g["grad/" + n]) for n, _ in params if "grad/" + n in g.files}
    check_grads_calibrated(params, g32, g64, g["grad_norms"])


def test_gan_iteration_matches_reference():
    """GAN_LAMBDA 1: one adversarial_train iteration — generator
    losses with the LSGAN terms through both discriminators, generator gradients, the
    D step's losses and discriminator gradients, discriminator running statistics."""
    from vae2.model import FullModel_D
    from vae2.optim import FusedAdam
    g = golden("tiny_gan")
    fm = hip_model(dict(arch="tiny"), with_d=True, gan_lambda=1.0)
    ed, ez, ds, df = fm.encdec_model, fm.encz_model, fm.D_model_sequence, fm.D_model_frame
    opt_g = FusedAdam([ez, ed], lr=1e-4)
    opt_d = FusedAdam([ds, df], lr=1e-4)
    xt, x2t, x3t = (t(g[k]).to(DEV) for k in ("xt", "x2t", "x3t"))
    fm.set_noise(t(g["eps"]), t(g["code"]))
    opt_g.zero_grad()
    losses, x1p, x2p, x3p = fm(xt, x2t, x3t, 1.0)
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL", "gan_seq", "gan_frame"]
    for n, v in zip(names, losses):
        ref = float(g["loss_" + n])
        assert abs(float(v.reshape(-1)[0]) - ref) <= 1e-5 * abs(ref) + 1e-7, (n, float(v), ref)
    opt_d.zero_grad()
    losses[0].backward()
    torch.cuda.synchronize()
    # no discriminator weight gradient is computed in the generator pass
    assert all(float(p.main_grad.abs().max()) == 0.0 for _, p in named_params(("ds", ds),
                                                                              ("df", df)))
    gparams = named_params(("encz", ez), ("ed", ed))
    g64 = oracle_elbo_grads(dict(arch="tiny"), g, torch.float64, with_d=True, gan_lambda=1.0,
                            d_step=True)
    check_grads_calibrated(gparams, {n: t(g["grad/" + n]) for n, _ in gparams}, g64,
                           g["grad_norms"])
    opt_g.step()
    fmd = FullModel_D(ds, df, None).to(DEV)
    dl = fmd(x2t, x2p.detach())
    for n, v in zip(("D_all", "D_seq", "D_frame"), dl):
        ref = float(g["loss_" + n])
        assert abs(float(v.reshape(-1)[0]) - ref) <= 1e-5 * abs(ref), (n, float(v), ref)
    opt_d.zero_grad()
    dl[0].backward()
    torch.cuda.synchronize()
    # The discriminator head is discontinuous at its ReLU: on the real clip one pixel of
    # D_seq's head sits within 1e-6 (relative) of zero, so any fp32 forward may flip its
    # mask, which moves every D_seq gradient by up to 1.9e-2 relative.  Measured on the
    # fp64 oracle: 1e-6 relative input noise reproduces exactly that jump, and the fp64
    # oracle evaluated at the HIP path's own stage-4 features matches the HIP gradients
    # to 2e-6 (scripts/diag_head.py).  The reference's fp32 run happened to stay on the
    # fp64 side, so its spread (4e-6) cannot calibrate this: floor 2e-2.
    dparams = named_params(("ds", ds), ("df", df))
    check_grads_calibrated(dparams, {n: t(g["dgrad/" + n]) for n, _ in dparams}, g64,
                           g["dgrad_norms"], floor=2e-2)
    opt_d.step()
    rs = {("ds." + k): v for k, v in ds.state_dict().items() if "running" in k}
    rs.update({("df." + k): v for k, v in df.state_dict().items() if "running" in k})
    rsum = np.array([float(rs[k].double().sum()) for k in sorted(rs)])
    np.testing.assert_allclose(rsum, g["d_running_sum"], rtol=1e-4, atol=1e-4)


def test_w18_backward_matches_reference():
    """Production-width kernels (W18: 18/36/72/144-channel branches, 64-channel stems,
    270-channel heads) in the backward, on the reference's golden case (32x32, B=2):
    every per-parameter gradient against the fp64 oracle with the calibrated rule and
    every gradient norm against the reference's own (tests/golden/w18.npz)."""
    kw = dict(arch="w18")
    g = golden("w18")
    fm = hip_model(kw)
    fm.set_noise(t(g["eps"]), t(g["code"]))
    losses = fm(t(g["xt"]).to(DEV), t(g["x2t"]).to(DEV), t(g["x3t"]).to(DEV), 1.0)[0]
    losses[0].backward()
    torch.cuda.synchronize()
    params = named_params(("encz", fm.encz_model), ("ed", fm.encdec_model))
    assert [n for n, _ in params] == list(g["grad_names"])
    g64 = oracle_elbo_grads(kw, g, torch.float64)
    g32 = oracle_elbo_grads(kw, g, torch.float32)  # the reference's ops in fp32 (pinned)
    ref_norms = np.asarray(g["grad_norms"])
    o32 = np.array([float(g32[n].double().norm()) for n, _ in params])
    big = ref_norms > 1e-6 * ref_norms.max()
    assert np.median(np.abs(o32[big] - ref_norms[big]) / ref_norms[big]) < 1e-2
    check_grads_calibrated(params, g32, g64, ref_norms)


def test_w18_backward_64x128_matches_fp64_oracle():
    """W18 backward at 64x128 (B=2): more pixels per BN channel, the K-split and
    stride-parity dgrad instances of the larger layers."""
    kw = dict(arch="w18", hw=(64, 128))
    gen = torch.Generator().manual_seed(5)
    xs = [torch.randn(2, 9, 64, 128, generator=gen) for _ in range(3)]
    eps = torch.randn(2, 10, 1, 1, generator=gen)
    code = torch.randn(2, 10, 1, 1, generator=gen)
    fm = hip_model(kw)
    fm.set_noise(eps, code)
    losses = fm(*[x.to(DEV) for x in xs], 1.0)[0]
    losses[0].backward()
    torch.cuda.synchronize()
    params = named_params(("encz", fm.encz_model), ("ed", fm.encdec_model))
    g64 = oracle_elbo_grads(kw, None, torch.float64, xs=xs, noise_=(eps, code))
    g32 = oracle_elbo_grads(kw, None, torch.float32, xs=xs, noise_=(eps, code))
    check_grads_calibrated(params, g32, g64)


def test_w18_gather_remainder_form_gradients_vs_fp64():
    """The shipped default of the gather GEMM (set_tune key 6 = 2: 18-output-channel convs as
    16 MFMA + 2 VALU channels) against the plain form (key 6 = 0) on identical inputs: both
    sets of W18 gradients pass the calibrated fp64-oracle rule, and the remainder form is
    not further from fp64 than the plain one (median per-tensor distance within 1.5x), so
    the 5 % step-1 trajectory difference between the two forms (tests/test_bf16_gpu.py) is
    summation order amplified by Adam's first steps, not an error of the remainder path."""
    from vae2 import _lib
    lib = _lib.load()
    kw = dict(arch="w18", hw=(64, 128))
    gen = torch.Generator().manual_seed(9)
    xs = [torch.randn(2, 9, 64, 128, generator=gen) for _ in range(3)]
    eps = torch.randn(2, 10, 1, 1, generator=gen)
    code = torch.randn(2, 10, 1, 1, generator=gen)
    g64 = oracle_elbo_grads(kw, None, torch.float64, xs=xs, noise_=(eps, code))
    g32 = oracle_elbo_grads(kw, None, torch.float32, xs=xs, noise_=(eps, code))
    med = {}
    for form in (0, 2):
        prev = lib.vae2_conv2d_set_tune(6, form)
        assert prev >= 0
        try:
            fm = hip_model(kw)
            fm.set_noise(eps, code)
            losses = fm(*[x.to(DEV) for x in xs], 1.0)[0]
            losses[0].backward()
            torch.cuda.synchronize()
            params = named_params(("encz", fm.encz_model), ("ed", fm.encdec_model))
            med[form], _ = check_grads_calibrated(params, g32, g64)
        finally:
            lib.vae2_conv2d_set_tune(6, prev)
    print("median per-tensor distance to fp64: plain", med[0], "remainder", med[2])
    assert med[2] <= 1.5 * med[0] + 1e-6, med


def test_bench_geometry_forward_matches_oracle():
    """The benchmark's exact geometry (128x256, B=8): loss and x2t_hat against the
    oracle (kernel instances and BN statistics at the bench's batch)."""
    from oracle import ref_cpu
    kw = dict(arch="w18", hw=(128, 256))
    ed, ez = build(make_cfg(**kw))
    ed_c, ez_c = copy.deepcopy(ed), copy.deepcopy(ez)
    gen = torch.Generator().manual_seed(3)
    xs = [torch.randn(8, 9, 128, 256, generator=gen) for _ in range(3)]
    eps = torch.randn(8, 10, 1, 1, generator=gen)
    code = torch.randn(8, 10, 1, 1, generator=gen)
    with torch.no_grad():
        terms, preds, _ = ref_cpu.elbo(ez_c, ed_c, *xs, eps, code)
    from vae2.model import FullModel_encdec
    fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0, 0.0).to(DEV)
    fm.set_noise(eps, code)
    with torch.no_grad():
        losses, x1p, x2p, x3p = fm(*[x.to(DEV) for x in xs], 1.0)
    ref = float(terms["loss_all"])
    assert abs(float(losses[0]) - ref) <= 1e-5 * abs(ref)
    assert max_rel(x2p, preds[1]) < 1e-4
    assert max_rel(x3p, preds[2]) < 1e-3


def test_deferred_nonfinite_check_raises():
    """MI355X.DEFER_CHECKS: a NaN reaching the predictions is reported at
    check_anomalies() with the reference's AssertionError (utils.py:63-65)."""
    fm = hip_model(dict(arch="tiny"))
    fm.defer_checks = True
    g = golden("tiny_native")
    fm.set_noise(t(g["eps"]), t(g["code"]))
    xt = t(g["xt"]).clone()
    xt[0, 0, 0, 0] = float("nan")
    with torch.no_grad():
        fm(xt.to(DEV), t(g["x2t"]).to(DEV), t(g["x3t"]).to(DEV), 1.0)
    with pytest.raises(AssertionError, match="nan or inf"):
        fm.check_anomalies()


def test_bench_geometry_grouped_convs_are_exact():
    """At the benchmark's geometry (128x256, B=8: the lower branches' direct-3x3 convs
    share launches per depth level) the training step with grouped conv launches equals
    the step with every conv on its own launch bit for bit (loss, predictions, every
    gradient)."""
    from vae2 import _lib
    from vae2.model import FullModel_encdec
    from vae2.optim import FusedAdam
    lib = _lib.load()
    gen = torch.Generator().manual_seed(4)
    xs = [torch.randn(8, 9, 128, 256, generator=gen).to(DEV) for _ in range(3)]
    eps = torch.randn(8, 10, 1, 1, generator=gen)
    code = torch.randn(8, 10, 1, 1, generator=gen)
    out = []
    prev = lib.vae2_conv2d_set_grouping(1)
    try:
        for on in (1, 0):
            lib.vae2_conv2d_set_grouping(on)
            ed, ez = build(make_cfg(arch="w18", hw=(128, 256)))
            fm = FullModel_encdec(ez, ed, None, None, None, None, None, 1.0, 0.1, 1.0,
                                  0.0).to(DEV)
            opt = FusedAdam([fm.encz_model, fm.encdec_model], lr=1e-4)
            fm.set_noise(eps, code)
            opt.zero_grad()
            losses, _, x2p, _ = fm(*xs, 1.0)
            losses[0].backward()
            torch.cuda.synchronize()
            out.append((float(losses[0]), x2p.detach().cpu(),
                        torch.cat([f.grad for f in opt.flats]).cpu()))
    finally:
        lib.vae2_conv2d_set_grouping(prev)
    (l1, p1, g1), (l0, p0, g0) = out
    assert l1 == l0
    assert torch.equal(p1, p0)
    assert torch.equal(g1, g0)


def test_vaegan_baseline_matches_reference():
    """IS_BASELINE + VAE_GAN (utils.py:132-141): L1(x2t_hat, x3t) + KL + both LSGAN terms
    on x2t_hat with the decoders under no_grad, and the D step on x3t as the real sample
    (function.py:503-504, vae2.trainer): losses, generator and discriminator gradients."""
    from vae2.model import FullModel_D
    kw = dict(arch="tiny", baseline=True, mode="VAE_GAN")
    g = golden("tiny_vaegan")
    fm = hip_model(kw, with_d=True, gan_lambda=1.0)
    ed, ez, ds, df = fm.encdec_model, fm.encz_model, fm.D_model_sequence, fm.D_model_frame
    xt, x2t, x3t = (t(g[k]).to(DEV) for k in ("xt", "x2t", "x3t"))
    fm.set_noise(t(g["eps"]), t(g["code"]))
    losses, x1p, x2p, x3p = fm(xt, x2t, x3t, 1.0, is_baseline=True, baseline_mode="VAE_GAN")
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL", "gan_seq", "gan_frame"]
    for n, v in zip(names, losses):
        ref = float(g["loss_" + n])
        got = float(v.reshape(-1)[0]) if torch.is_tensor(v) else float(v)
        assert abs(got - ref) <= 1e-5 * abs(ref) + 1e-7, (n, got, ref)
    assert max_rel(x2p, t(g["x2p"])) < 1e-4
    losses[0].backward()
    torch.cuda.synchronize()
    g64 = oracle_elbo_grads(kw, g, torch.float64, with_d=True, gan_lambda=1.0, d_step=True)
    # the generator gradient reaches the encoder through both discriminators (ReLU masks
    # at rounding distance, as in the GAN test): calibrate with the fp64 sensitivity too
    g64p = [oracle_elbo_grads(kw, g, torch.float64, with_d=True, gan_lambda=1.0, perturb=1e-6,
                              pseed=s) for s in range(4)]
    gparams = named_params(("encz", ez), ("ed", ed))
    check_grads_calibrated(gparams, {n: t(g["grad/" + n]) for n, _ in gparams
                                     if "grad/" + n in g.files}, g64, g["grad_norms"], g64p=g64p)
    fmd = FullModel_D(ds, df, None).to(DEV)
    dl = fmd(x3t, x2p.detach())
    for n, v in zip(("D_all", "D_seq", "D_frame"), dl):
        ref = float(g["loss_" + n])
        assert abs(float(v.reshape(-1)[0]) - ref) <= 1e-5 * abs(ref), (n, float(v), ref)
    for m in (ds, df):
        from vae2.params import flatten
        flatten(m).zero_grad()
    dl[0].backward()
    torch.cuda.synchronize()
    # the discriminator head's ReLU mask can flip within fp32 noise (see the GAN test)
    dparams = named_params(("ds", ds), ("df", df))
    check_grads_calibrated(dparams, {n: t(g["dgrad/" + n]) for n, _ in dparams}, g64,
                           g["dgrad_norms"], floor=2e-2)


def test_eval_prior_sampling_matches_reference():
    """The evaluation forward (function.py:60,124-136; tools/inference.py): eval() —
    every BatchNorm on its running statistics (vae2_bn_eval_coeffs, the heads' eval path,
    the discriminators in the GAN terms) — prior sampling, no_grad, on a trained-looking
    state (tests/golden/tiny_eval.npz).  No batch statistics couple the layers, so the
    predictions hold 1e-4 max-relative end to end."""
    g = golden("tiny_eval")
    fm = hip_model(dict(arch="tiny"), with_d=True, gan_lambda=1.0)
    load_eval_state(g, (fm.encz_model, fm.encdec_model, fm.D_model_sequence, fm.D_model_frame))
    fm.eval()
    fm.set_noise(t(g["eps"]), t(g["code"]))
    with torch.no_grad():
        losses, x1p, x2p, x3p = fm(t(g["xt"]).to(DEV), t(g["x2t"]).to(DEV), t(g["x3t"]).to(DEV),
                                   1.0, sampling_mode="prior_sampling")
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL", "gan_seq", "gan_frame"]
    for n, v in zip(names, losses):
        ref = float(g["loss_" + n])
        got = float(v.reshape(-1)[0]) if torch.is_tensor(v) else float(v)
        assert abs(got - ref) <= 1e-5 * abs(ref) + 1e-7, (n, got, ref)
    for k, p in (("x1p", x1p), ("x2p", x2p), ("x3p", x3p)):
        assert max_rel(p, t(g[k])) < 1e-4, k


def test_reference_checkpoint_resumes():
    """A checkpoint the reference wrote (train.py:320-324) loaded into the HIP model and
    FusedAdam (torch.optim.Adam state format): the next step's loss terms equal the
    reference's (1e-5) and, after the Adam update from the saved moments, the parameters
    are no further from an fp64 oracle run than the reference's fp32 ones (x3, median)."""
    from oracle import ref_cpu
    from vae2.optim import FusedAdam
    ck = ref_checkpoint()
    g = golden("ref_ckpt")
    fm = hip_model(dict(arch="tiny"), with_d=True, gan_lambda=0.0)
    fm.load_state_dict({k: v.to(DEV) for k, v in ck["state_dict"].items()}, strict=True)
    ez, ed = fm.encz_model, fm.encdec_model
    opt = FusedAdam([ez, ed], lr=1e-4)
    opt.load_state_dict(ck["optimizer_encdec"])
    assert opt.step_count == 1
    fm.set_noise(t(g["eps"]), t(g["code"]))
    opt.zero_grad()
    losses = fm(t(g["xt"]).to(DEV), t(g["x2t"]).to(DEV), t(g["x3t"]).to(DEV), 1.0)[0]
    for n, v in zip(["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL"], losses[:5]):
        ref = float(g["loss_" + n])
        assert abs(float(v.reshape(-1)[0]) - ref) <= 1e-5 * abs(ref) + 1e-7, (n, float(v), ref)
    losses[0].backward()
    opt.step()
    torch.cuda.synchronize()
    named = named_params(("encz_model", ez), ("encdec_model", ed))
    psum = np.array([float(p.detach().double().sum()) for _, p in sorted(named)])
    # fp64 oracle from the same checkpoint
    ed64, ez64, ds64, df64 = build(make_cfg("tiny"), with_d=True)
    from vae2.model import FullModel_encdec
    f64 = FullModel_encdec(ez64, ed64, ds64, df64, None, None, None, 1.0, 0.1, 1.0, 0.0)
    f64.load_state_dict(ck["state_dict"])
    f64.double()
    n64 = [(n, p) for n, p in f64.named_parameters() if "D_model" not in n]
    o64 = torch.optim.Adam([{"params": [p for _, p in n64]}], lr=1e-4)
    o64.load_state_dict(ck["optimizer_encdec"])
    terms, _, _ = ref_cpu.elbo(ez64, ed64, *[t(g[k]).double() for k in ("xt", "x2t", "x3t")],
                               t(g["eps"]).double(), t(g["code"]).double())
    terms["loss_all"].backward()
    o64.step()
    assert [n for n, _ in sorted(n64)] == [n for n, _ in sorted(named)] == list(g["param_names"])
    p64 = np.array([float(p.detach().sum()) for _, p in sorted(n64)])
    d_ref = np.abs(g["param_sum"] - p64)
    d_hip = np.abs(psum - p64)
    assert np.median(d_hip) <= 3 * np.median(d_ref) + 1e-9, (np.median(d_hip), np.median(d_ref))
