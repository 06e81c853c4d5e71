"""Pin the CPU oracle (oracle/ref_cpu.py) to golden vectors produced by the
reference itself (tests/golden/make_golden.py), and check seeded-init parity of
the vae2 model trees against the reference's init checksums."""
import numpy as np
import pytest
import torch

from helpers import (build, checksums, golden, load_eval_state, make_cfg, max_rel, ref_checkpoint,
                     rel, t)
from oracle import ref_cpu

CASES = {
    "tiny_native": dict(arch="tiny"),
    "tiny_hdz": dict(arch="tiny", hd=True, z=3),
    "tiny_base": dict(arch="tiny", baseline=True),
    "w18": dict(arch="w18"),
}


def _noise(g, hd):
    if hd:
        eps = [t(g[f"eps{i}"]) for i in range(4)]
    else:
        eps = t(g["eps"])
    return eps, t(g["code"])


@pytest.mark.parametrize("case", list(CASES))
def test_init_parity(case):
    g = golden(case)
    ed, ez = build(make_cfg(**CASES[case]))
    s, a = checksums(ed.state_dict())
    np.testing.assert_array_equal(s, g["init_ed_sum"])
    np.testing.assert_array_equal(a, g["init_ed_abs"])
    s, a = checksums(ez.state_dict())
    np.testing.assert_array_equal(s, g["init_ez_sum"])
    np.testing.assert_array_equal(a, g["init_ez_abs"])


@pytest.mark.parametrize("case", list(CASES))
def test_oracle_forward_matches_reference(case):
    torch.set_num_threads(8)
    kw = CASES[case]
    g = golden(case)
    ed, ez = build(make_cfg(**kw))
    ed.train(), ez.train()
    eps, code = _noise(g, kw.get("hd", False))
    terms, (x1p, x2p, x3p), aux = ref_cpu.elbo(
        ez, ed, t(g["xt"]), t(g["x2t"]), t(g["x3t"]), eps, code,
        is_baseline=kw.get("baseline", False))
    for name, v in terms.items():
        ref = float(g["loss_" + name])
        assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-7, (name, float(v), ref)
    assert max_rel(x2p, t(g["x2p"])) < 1e-4
    # decoders sit ~300 BN layers deeper: the reference's own fp32 spread is ~5e-4 (App. D)
    assert rel(x3p, t(g["x3p"])) < 1e-3
    assert rel(x1p, t(g["x1p"])) < 1e-3
    if not kw.get("hd", False):
        assert max_rel(aux["muvar"], t(g["muvar"])) < 1e-4


def test_oracle_grads_and_adam_match_reference():
    torch.set_num_threads(8)
    g = golden("tiny_native")
    ed, ez = build(make_cfg("tiny"))
    eps, code = _noise(g, False)
    xt, x2t, x3t = t(g["xt"]), t(g["x2t"]), t(g["x3t"])
    terms, _, _ = ref_cpu.elbo(ez, ed, xt, x2t, x3t, eps, code)
    terms["loss_all"].backward()
    params = list(ez.named_parameters(prefix="encz")) + list(ed.named_parameters(prefix="ed"))
    names = list(g["grad_names"])
    assert names == [n for n, _ in params]
    norms = np.array([float(p.grad.double().norm()) for _, p in params])
    ref_norms = g["grad_norms"]
    big = ref_norms > 1e-6 * ref_norms.max()  # analytically-zero biases before BN excluded
    np.testing.assert_allclose(norms[big], ref_norms[big], rtol=1e-3)
    for n, p in params:
        key = "grad/" + n
        if key in g.files and np.abs(g[key]).max() > 1e-6 * ref_norms.max():
            assert rel(p.grad, t(g[key])) < 1e-3, n
    # Adam trajectory (reference: torch.optim.Adam lr 1e-4, train.py:251-261)
    opt = torch.optim.Adam([{"params": [p for _, p in params]}], lr=1e-4)
    opt.step()
    traj = []
    for k in range(1, 3):
        opt.zero_grad()
        torch.manual_seed(200 + k)
        e = torch.randn(2, 4, 1, 1)
        c = torch.randn(2, 4, 1, 1)
        terms, _, _ = ref_cpu.elbo(ez, ed, xt, x2t, x3t, e, c)
        traj.append(float(terms["loss_all"]))
        terms["loss_all"].backward()
        opt.step()
    np.testing.assert_allclose(traj, g["adam_losses"], rtol=1e-5)
    psum = np.array([float(p.detach().double().sum()) for _, p in sorted(params)])
    np.testing.assert_allclose(psum, g["adam_param_sum"], rtol=1e-4, atol=1e-6)


# ---- ELBO modes and the GAN step (fixtures: make_golden.py tiny_anneal / tiny_det /
# tiny_prior / tiny_gan) ----
MODES = {
    "tiny_anneal": dict(kw=dict(arch="tiny", mode="VAE_ANNEAL"), multiplier=0.37),
    "tiny_det": dict(kw=dict(arch="tiny", baseline=True, mode="DETERMINISTIC")),
    "tiny_prior": dict(kw=dict(arch="tiny"), prior=True),
}


def _grad_check(params, g, prefix="grad"):
    ref_norms = g[prefix + "_norms"]
    big = ref_norms > 1e-6 * ref_norms.max()  # analytically-zero biases before BN excluded
    norms = np.array([float(p.grad.double().norm()) if p.grad is not None else 0.0
                      for _, p in params])
    np.testing.assert_allclose(norms[big], ref_norms[big], rtol=1e-3)
    for n, p in params:
        key = f"{prefix}/{n}"
        if key in g.files and np.abs(g[key]).max() > 1e-6 * ref_norms.max():
            assert rel(p.grad, t(g[key])) < 1e-3, n


@pytest.mark.parametrize("case", list(MODES))
def test_oracle_modes_match_reference(case):
    """VAE_ANNEAL (KL x multiplier), DETERMINISTIC (baseline, no posterior net) and
    prior sampling (z drawn from N(0, I)): loss terms, predictions and gradients."""
    torch.set_num_threads(8)
    spec = MODES[case]
    kw = spec["kw"]
    g = golden(case)
    ed, ez = build(make_cfg(**kw))
    det = kw.get("mode") == "DETERMINISTIC"
    assert (ez is None) == det
    s, a = checksums(ed.state_dict())
    np.testing.assert_array_equal(s, g["init_ed_sum"])
    eps = None if det else t(g["eps"])
    code = None if det else t(g["code"])
    xt, x2t, x3t = t(g["xt"]), t(g["x2t"]), t(g["x3t"])
    terms, (x1p, x2p, x3p), _ = ref_cpu.elbo(
        ez, ed, xt, x2t, x3t, eps, code, multiplier=spec.get("multiplier", 1.0),
        is_baseline=kw.get("baseline", False), baseline_mode=kw.get("mode", "VAE_NATIVE"),
        prior=spec.get("prior", False))
    for name, v in terms.items():
        ref = float(g["loss_" + name])
        assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-7, (name, float(v), ref)
    assert max_rel(x2p, t(g["x2p"])) < 1e-4
    terms["loss_all"].backward()
    params = (list(ez.named_parameters(prefix="encz")) if ez is not None else []) + \
        list(ed.named_parameters(prefix="ed"))
    assert list(g["grad_names"]) == [n for n, _ in params]
    _grad_check(params, g)


def test_oracle_gan_iteration_matches_reference():
    """One full adversarial_train iteration with GAN_LAMBDA 1 (function.py:491-512):
    G losses incl. the LSGAN terms, G gradients, Adam, D losses, D gradients, Adam,
    discriminator running statistics and parameter sums."""
    torch.set_num_threads(8)
    g = golden("tiny_gan")
    ed, ez, ds, df = build(make_cfg("tiny"), with_d=True)
    for key, m in (("ds", ds), ("df", df)):
        s, a = checksums(m.state_dict())
        np.testing.assert_array_equal(s, g[f"init_{key}_sum"])
        np.testing.assert_array_equal(a, g[f"init_{key}_abs"])
    for m in (ed, ez, ds, df):
        m.train()
    xt, x2t, x3t = t(g["xt"]), t(g["x2t"]), t(g["x3t"])
    terms, (x1p, x2p, x3p), _ = ref_cpu.elbo(ez, ed, xt, x2t, x3t, t(g["eps"]), t(g["code"]),
                                             ds=ds, df=df, gan_lambda=1.0)
    for name, v in terms.items():
        ref = float(g["loss_" + name])
        assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-7, (name, float(v), ref)
    gparams = list(ez.named_parameters(prefix="encz")) + list(ed.named_parameters(prefix="ed"))
    opt_g = torch.optim.Adam([p for _, p in gparams], lr=1e-4)
    opt_g.zero_grad()
    terms["loss_all"].backward()
    _grad_check(gparams, g)
    opt_g.step()
    dparams = list(ds.named_parameters(prefix="ds")) + list(df.named_parameters(prefix="df"))
    assert list(g["dgrad_names"]) == [n for n, _ in dparams]
    opt_d = torch.optim.Adam([p for _, p in dparams], lr=1e-4)
    dl = ref_cpu.d_losses(ds, df, x2t, x2p)
    for name, v in zip(("D_all", "D_seq", "D_frame"), dl):
        ref = float(g["loss_" + name])
        assert abs(float(v.reshape(-1)[0]) - ref) <= 1e-5 * abs(ref), (name, float(v), ref)
    opt_d.zero_grad()
    dl[0].backward()
    _grad_check(dparams, g, "dgrad")
    opt_d.step()
    rs = {("ds." + k): v for k, v in ds.state_dict().items() if "running" in k}
    rs.update({("df." + k): v for k, v in df.state_dict().items() if "running" in k})
    # running means of the discriminators sum to ~1e-5 (cancellation): absolute floor
    np.testing.assert_allclose(checksums(rs)[0], g["d_running_sum"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(checksums({n: p.detach() for n, p in gparams})[0],
                               g["g_param_sum"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(checksums({n: p.detach() for n, p in dparams})[0],
                               g["d_param_sum"], rtol=1e-4, atol=1e-6)


def test_oracle_vaegan_baseline_matches_reference():
    """IS_BASELINE + VAE_GAN (utils.py:132-141): L1(x2t_hat, x3t) + KL + both LSGAN terms,
    decoders under no_grad; the D step's real sample is x3t (function.py:503-504)."""
    torch.set_num_threads(8)
    g = golden("tiny_vaegan")
    ed, ez, ds, df = build(make_cfg("tiny", baseline=True, mode="VAE_GAN"), with_d=True)
    xt, x2t, x3t = t(g["xt"]), t(g["x2t"]), t(g["x3t"])
    terms, (x1p, x2p, x3p), _ = ref_cpu.elbo(ez, ed, xt, x2t, x3t, t(g["eps"]), t(g["code"]),
                                             is_baseline=True, baseline_mode="VAE_GAN",
                                             ds=ds, df=df, gan_lambda=1.0)
    for name, v in terms.items():
        ref = float(g["loss_" + name])
        assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-7, (name, float(v), ref)
    assert max_rel(x2p, t(g["x2p"])) < 1e-4
    gparams = list(ez.named_parameters(prefix="encz")) + list(ed.named_parameters(prefix="ed"))
    opt_g = torch.optim.Adam([p for _, p in gparams], lr=1e-4)
    terms["loss_all"].backward()
    _grad_check(gparams, g)
    assert all(p.grad is None for n, p in gparams if n.startswith("ed.dec"))  # no_grad decoders
    opt_g.step()
    dparams = list(ds.named_parameters(prefix="ds")) + list(df.named_parameters(prefix="df"))
    for p in (p for _, p in dparams):
        p.grad = None
    dl = ref_cpu.d_losses(ds, df, x3t, x2p)
    for name, v in zip(("D_all", "D_seq", "D_frame"), dl):
        ref = float(g["loss_" + name])
        assert abs(float(v.reshape(-1)[0]) - ref) <= 1e-5 * abs(ref), (name, float(v), ref)
    dl[0].backward()
    _grad_check(dparams, g, "dgrad")


def test_oracle_eval_prior_sampling_matches_reference():
    """Evaluation forward (function.py:60,124-136): eval() BatchNorm on running statistics
    (discriminators too), prior sampling, no_grad."""
    torch.set_num_threads(8)
    g = golden("tiny_eval")
    ed, ez, ds, df = build(make_cfg("tiny"), with_d=True)
    load_eval_state(g, (ez, ed, ds, df))
    for m in (ed, ez, ds, df):
        m.eval()
    with torch.no_grad():
        terms, (x1p, x2p, x3p), _ = ref_cpu.elbo(ez, ed, t(g["xt"]), t(g["x2t"]), t(g["x3t"]),
                                                 t(g["eps"]), t(g["code"]), prior=True,
                                                 ds=ds, df=df, gan_lambda=1.0)
    for name, v in terms.items():
        ref = float(g["loss_" + name])
        assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-7, (name, float(v), ref)
    for k, p in (("x1p", x1p), ("x2p", x2p), ("x3p", x3p)):
        assert max_rel(p, t(g[k])) < 1e-5, k


def test_reference_checkpoint_interchange():
    """A checkpoint the reference itself wrote (train.py:320-324: epoch / state_dict /
    optimizer_encdec) loads strictly into this package's FullModel_encdec tree, and the
    oracle's next step from it (loss terms, torch Adam from the saved moments) is the
    reference's (tests/golden/ref_ckpt.npz)."""
    torch.set_num_threads(8)
    from vae2.model import FullModel_encdec
    ck = ref_checkpoint()
    assert ck["epoch"] == 1 and set(ck) == {"epoch", "state_dict", "optimizer_encdec"}
    ed, ez, ds, df = build(make_cfg("tiny"), with_d=True)
    fm = FullModel_encdec(ez, ed, ds, df, None, None, None, 1.0, 0.1, 1.0, 0.0)
    assert list(fm.state_dict()) == list(ck["state_dict"])
    fm.load_state_dict(ck["state_dict"], strict=True)
    g = golden("ref_ckpt")
    named = [(n, p) for n, p in fm.named_parameters() if "D_model" not in n]
    assert len(ck["optimizer_encdec"]["state"]) == len(named)
    opt = torch.optim.Adam([{"params": [p for _, p in named]}], lr=1e-4)
    opt.load_state_dict(ck["optimizer_encdec"])
    terms, _, _ = ref_cpu.elbo(ez, ed, t(g["xt"]), t(g["x2t"]), t(g["x3t"]), t(g["eps"]),
                               t(g["code"]))
    for name in ("loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL"):
        ref = float(g["loss_" + name])
        assert abs(float(terms[name]) - ref) <= 1e-5 * abs(ref) + 1e-7, (name, ref)
    opt.zero_grad()
    terms["loss_all"].backward()
    opt.step()
    assert [n for n, _ in sorted(named)] == list(g["param_names"])
    np.testing.assert_allclose(checksums({n: p.detach() for n, p in named})[0], g["param_sum"],
                               rtol=1e-4, atol=1e-6)
