"""Generate the golden vectors that pin oracle/ref_cpu.py to the reference.

Runs ONLY in the build container, where /root/reference exists: it imports the
reference's own modules (lib/models/enc_hrnet.py, lib/utils/utils.py,
lib/core/criterion.py) read-only, with the two shims SURVEY.md App. C lists
(numpy.int alias, an attribute-dict config instead of yacs), and writes data
only (inputs, noise, outputs, loss terms, gradients, checksums) as .npz here.
Nothing from the reference is copied.

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz (+ the .pth.tar)

Cases
  tiny_native   tiny HRNet, 32x32, B=2, L=3, Z=4, VAE_NATIVE:
                inputs, eps/code, mu|logvar, z, x2t/x3t/xt predictions, loss terms,
                every parameter gradient, 3 Adam steps (loss trajectory + param sums)
  tiny_hdz      same with HD_Z (Z_DIM 3)
  tiny_base     IS_BASELINE=True, VAE_NATIVE (decoders under no_grad, L1(x2t_hat, x3t))
  w18           HRNet-W18-small-v2, 32x32, B=2, Z=10: outputs, losses, per-parameter
                gradient norms, init checksums (weights regenerate from the seed)
  tiny_anneal   VAE_ANNEAL with multiplier 0.37 (KL weight = X3RECON_LAMBDA * multiplier,
                utils.py:74), full gradients
  tiny_det      IS_BASELINE + DETERMINISTIC (no posterior net, no code maps, KL = 0;
                utils.py:76,102-103,128-131; train.py:80 builds no encz), full gradients
  tiny_prior    sampling_mode='prior_sampling' (z ~ N(0, I) drawn in place of eps,
                utils.py:88-89,97-98), full gradients
  tiny_gan      GAN_LAMBDA 1: one full adversarial_train iteration (function.py:491-512):
                G step with the LSGAN terms through both discriminators (utils.py:114-119),
                Adam, then the D step (FullModel_D, utils.py:256-276) and its Adam;
                G and D gradients, D losses, running statistics, parameter sums
  tiny_vaegan   IS_BASELINE + VAE_GAN: L1(x2t_hat, x3t) + KL + both LSGAN terms on x2t_hat
                (utils.py:132-141), decoders under no_grad; the D step takes x3t as the real
                sample (function.py:503-504)
  tiny_eval     evaluation forward (function.py:60,124-136): model_encdec.eval() (BatchNorm
                on running statistics, discriminators included), sampling_mode
                'prior_sampling', no_grad, on a trained-looking state (Kaiming-scale conv
                weights, random BN affine and running statistics, stored as sd/<key>)
  ref_ckpt      a checkpoint the reference itself writes (train.py:320-324 format:
                epoch / state_dict / optimizer_encdec, torch.save) after one Adam step,
                -> ref_checkpoint_encdec.pth.tar; ref_ckpt.npz holds the next training
                step taken from that state (noise, loss terms, parameter sums after Adam)

    python tests/golden/make_golden.py [case ...]   # default: all cases
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/lib"


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)


def stages(tiny):
    if tiny:
        return {"STAGE1": dict(NUM_MODULES=1, NUM_BRANCHES=1, BLOCK="BOTTLENECK", NUM_BLOCKS=[1],
                               NUM_CHANNELS=[8], FUSE_METHOD="SUM"),
                "STAGE2": dict(NUM_MODULES=1, NUM_BRANCHES=2, BLOCK="BASIC", NUM_BLOCKS=[1, 1],
                               NUM_CHANNELS=[4, 8], FUSE_METHOD="SUM"),
                "STAGE3": dict(NUM_MODULES=1, NUM_BRANCHES=3, BLOCK="BASIC",
                               NUM_BLOCKS=[1, 1, 1], NUM_CHANNELS=[4, 8, 16], FUSE_METHOD="SUM"),
                "STAGE4": dict(NUM_MODULES=1, NUM_BRANCHES=4, BLOCK="BASIC",
                               NUM_BLOCKS=[1, 1, 1, 1], NUM_CHANNELS=[4, 8, 16, 32],
                               FUSE_METHOD="SUM")}
    return {"STAGE1": dict(NUM_MODULES=1, NUM_BRANCHES=1, BLOCK="BOTTLENECK", NUM_BLOCKS=[2],
                           NUM_CHANNELS=[64], FUSE_METHOD="SUM"),
            "STAGE2": dict(NUM_MODULES=1, NUM_BRANCHES=2, BLOCK="BASIC", NUM_BLOCKS=[2, 2],
                           NUM_CHANNELS=[18, 36], FUSE_METHOD="SUM"),
            "STAGE3": dict(NUM_MODULES=3, NUM_BRANCHES=3, BLOCK="BASIC", NUM_BLOCKS=[2, 2, 2],
                           NUM_CHANNELS=[18, 36, 72], FUSE_METHOD="SUM"),
            "STAGE4": dict(NUM_MODULES=2, NUM_BRANCHES=4, BLOCK="BASIC",
                           NUM_BLOCKS=[2, 2, 2, 2], NUM_CHANNELS=[18, 36, 72, 144],
                           FUSE_METHOD="SUM")}


def make_cfg(tiny, hd=False, baseline=False, mode="VAE_NATIVE", z=None, L=3):
    extra = AttrDict(IS_BASELINE=baseline, BASELINE_MODE=mode, Z_DIM=z or (4 if tiny else 10),
                     HD_Z=hd, FINAL_CONV_KERNEL=1)
    for k, v in stages(tiny).items():
        extra[k] = AttrDict(v)
    return AttrDict(MODEL=AttrDict(NAME="enc_hrnet", PRETRAINED="", EXTRA=extra),
                    DATASET=AttrDict(NUM_CLASSES=3), TRAIN=AttrDict(CLIP_LENGTH=L, IMAGE_SIZE=[32, 32]))


def checksums(sd):
    names = sorted(sd)
    s = np.array([float(sd[k].double().sum()) for k in names])
    a = np.array([float(sd[k].double().abs().sum()) for k in names])
    return names, s, a


def run_case(tag, tiny, hd=False, baseline=False, mode="VAE_NATIVE", B=2, H=32, W=32,
             full_grads=False, adam_steps=0, z=None, multiplier=1.0, sampling="default",
             gan=0.0):
    import torch
    import models.enc_hrnet as eh
    from core.criterion import KLLoss, L1Loss, lsgan_adversarial_loss
    from utils.utils import FullModel_D, FullModel_encdec

    cfg = make_cfg(tiny, hd, baseline, mode, z=z)
    L = cfg.TRAIN.CLIP_LENGTH
    zc = cfg.MODEL.EXTRA.Z_DIM
    det = mode == "DETERMINISTIC"
    torch.manual_seed(0)  # construction order of train.py:79-82
    ed = eh.get_encdec_model(cfg)
    ez = eh.get_encz_model(cfg) if not det else None
    ds = eh.get_D_sequence_model(cfg)
    df = eh.get_D_frame_model(cfg)
    init_ed = {k: v.clone() for k, v in ed.state_dict().items()}
    init_ez = {k: v.clone() for k, v in ez.state_dict().items()} if ez is not None else {}
    init_ds = {k: v.clone() for k, v in ds.state_dict().items()}
    init_df = {k: v.clone() for k, v in df.state_dict().items()}
    fm = FullModel_encdec(ez, ed, ds, df, L1Loss(), KLLoss(), lsgan_adversarial_loss(),
                          1.0, 0.1, 1.0, gan)
    fm.train()
    g = torch.Generator().manual_seed(1)
    xt, x2t, x3t = [torch.randn(B, 3 * L, H, W, generator=g) for _ in range(3)]
    out = {"xt": xt, "x2t": x2t, "x3t": x3t}

    # capture every network's inputs/outputs with forward hooks
    cap = {}
    ed_fwd = ed.forward

    def ed_hook(x, z=None, is_baseline=False):
        cap["ed_in"] = x.detach().clone()
        cap["ed_z"] = ([t.detach().clone() for t in z] if isinstance(z, list)
                       else (z.detach().clone() if z is not None else None))
        r = ed_fwd(x, z=z, is_baseline=is_baseline)
        return r
    ed.forward = ed_hook
    if ez is not None:
        ez.register_forward_hook(lambda m, i, o: cap.__setitem__(
            "muvar", [t.detach().clone() for t in o] if isinstance(o, list) else o.detach().clone()))

    torch.manual_seed(123)
    losses, x1p, x2p, x3p = fm(xt, x2t, x3t, multiplier, is_baseline=baseline, baseline_mode=mode,
                               sampling_mode=sampling)
    # replay the draws (eps then code; SURVEY.md App. C, verified bit-exact)
    torch.manual_seed(123)
    if not det:
        if hd:
            eps = [torch.randn(B, zc, m.shape[2], m.shape[3]) for m in cap["muvar"]]
        else:
            eps = torch.randn(B, zc, 1, 1)  # in prior_sampling: z itself
        code = torch.randn(B, zc, 1, 1)
        out["code"] = code
    if not det:
        if hd:
            for i, e in enumerate(eps):
                out[f"eps{i}"] = e
                out[f"muvar{i}"] = cap["muvar"][i]
                out[f"z{i}"] = cap["ed_z"][i]
        else:
            out["eps"] = eps
            out["muvar"] = cap["muvar"]
            out["z"] = cap["ed_z"]
    out["x1p"], out["x2p"], out["x3p"] = x1p.detach(), x2p.detach(), x3p.detach()
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL", "gan_seq", "gan_frame"]
    for n, v in zip(names, losses):
        out["loss_" + n] = torch.as_tensor(float(v.reshape(-1)[0]) if torch.is_tensor(v) else v)
    losses[0].backward()
    params = [(n, p) for n, p in (list(ez.named_parameters(prefix="encz")) if ez is not None
                                  else []) + list(ed.named_parameters(prefix="ed"))]
    gnames = [n for n, p in params]
    gnorm = np.array([float(p.grad.double().norm()) if p.grad is not None else 0.0
                      for n, p in params])
    out["grad_norms"] = torch.as_tensor(gnorm)
    if full_grads:
        for n, p in params:
            if p.grad is not None:
                out["grad/" + n] = p.grad.detach().clone()
    # running statistics after one step
    rs = {("encz." + k): v for k, v in ez.state_dict().items() if "running" in k} if ez else {}
    rs.update({("ed." + k): v for k, v in ed.state_dict().items() if "running" in k})
    rn, rsum, rabs = checksums(rs)
    out["running_sum"] = torch.as_tensor(rsum)
    out["running_abs"] = torch.as_tensor(rabs)
    # init checksums (weights regenerate from torch.manual_seed(0))
    _, s1, a1 = checksums(init_ed)
    out["init_ed_sum"], out["init_ed_abs"] = torch.as_tensor(s1), torch.as_tensor(a1)
    if ez is not None:
        _, s2, a2 = checksums(init_ez)
        out["init_ez_sum"], out["init_ez_abs"] = torch.as_tensor(s2), torch.as_tensor(a2)
    if gan:
        for key, sd in (("ds", init_ds), ("df", init_df)):
            _, s3, a3 = checksums(sd)
            out[f"init_{key}_sum"], out[f"init_{key}_abs"] = torch.as_tensor(s3), torch.as_tensor(a3)
        # the D step's real sample: x2t, or x3t in baseline mode (function.py:503-504)
        real = x3t if baseline else x2t
        run_d_step(out, fm, ds, df, params, xt, real, x2p, lsgan_adversarial_loss, FullModel_D)
    if adam_steps:
        ps = [p for n, p in list(ez.named_parameters()) + list(ed.named_parameters())]
        opt = torch.optim.Adam([{"params": ps}], lr=1e-4)
        traj = []
        opt.step()  # step 1 uses the gradients computed above
        for k in range(1, adam_steps):
            opt.zero_grad()
            torch.manual_seed(200 + k)
            ls = fm(xt, x2t, x3t, 1.0, is_baseline=baseline, baseline_mode=mode)[0]
            traj.append(float(ls[0]))
            ls[0].backward()
            opt.step()
        out["adam_losses"] = torch.as_tensor(np.array(traj))
        pn, psum, pabs = checksums({n: p.detach() for n, p in params})
        out["adam_param_sum"] = torch.as_tensor(psum)
        out["adam_param_abs"] = torch.as_tensor(pabs)
    arrays = {k: v.detach().numpy().astype(np.float64 if v.dtype == torch.float64 else np.float32)
              if torch.is_tensor(v) else np.asarray(v) for k, v in out.items()}
    arrays["grad_names"] = np.array(gnames)
    arrays["running_names"] = np.array(rn)
    path = os.path.join(HERE, f"{tag}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def run_d_step(out, fm, ds, df, gparams, xt, real, x2p, lsgan, FullModel_D):
    """The rest of one adversarial_train iteration (function.py:499-512): Adam on the
    generator (encz + ED, 'D_model' excluded, train.py:251-256), then the D step with
    `real` as the real sample."""
    import torch
    opt_g = torch.optim.Adam([{"params": [p for _, p in gparams]}], lr=1e-4)
    opt_g.step()
    fmd = FullModel_D(ds, df, lsgan())
    fmd.train()
    dparams = list(ds.named_parameters(prefix="ds")) + list(df.named_parameters(prefix="df"))
    opt_d = torch.optim.Adam([{"params": [p for _, p in dparams]}], lr=1e-4)
    dl = fmd(x2t=real, x2t_predict=x2p.detach())
    for n, v in zip(("D_all", "D_seq", "D_frame"), dl):
        out["loss_" + n] = torch.as_tensor(float(v.reshape(-1)[0]))
    opt_d.zero_grad()
    dl[0].backward()
    out["dgrad_norms"] = torch.as_tensor(np.array([float(p.grad.double().norm())
                                                   for _, p in dparams]))
    for n, p in dparams:
        out["dgrad/" + n] = p.grad.detach().clone()
    opt_d.step()
    rs = {("ds." + k): v for k, v in ds.state_dict().items() if "running" in k}
    rs.update({("df." + k): v for k, v in df.state_dict().items() if "running" in k})
    _, rsum, _ = checksums(rs)
    out["d_running_sum"] = torch.as_tensor(rsum)
    _, gsum, _ = checksums({n: p.detach() for n, p in gparams})
    out["g_param_sum"] = torch.as_tensor(gsum)
    _, dsum, _ = checksums({n: p.detach() for n, p in dparams})
    out["d_param_sum"] = torch.as_tensor(dsum)
    out["dgrad_names"] = np.array([n for n, _ in dparams])


CASES = {
    "tiny_native": dict(tiny=True, full_grads=True, adam_steps=3),
    # Z_DIM 3: with 2*Z_DIM equal to a branch width the reference's HD_Z z-net has a
    # None projection and fails (enc_hrnet.py:1018-1019, :1106)
    "tiny_hdz": dict(tiny=True, hd=True, z=3),
    "tiny_base": dict(tiny=True, baseline=True),
    "w18": dict(tiny=False),
    "tiny_anneal": dict(tiny=True, mode="VAE_ANNEAL", multiplier=0.37, full_grads=True),
    # DETERMINISTIC is only runnable with IS_BASELINE (non-baseline reads mus, utils.py:113)
    "tiny_det": dict(tiny=True, baseline=True, mode="DETERMINISTIC", full_grads=True),
    "tiny_prior": dict(tiny=True, sampling="prior_sampling", full_grads=True),
    "tiny_gan": dict(tiny=True, gan=1.0, full_grads=True),
    "tiny_vaegan": dict(tiny=True, baseline=True, mode="VAE_GAN", gan=1.0, full_grads=True),
}


def _full_model(gan):
    """Tiny ED / EDz / D-seq / D-frame in train.py:79-82 order and FullModel_encdec."""
    import torch
    import models.enc_hrnet as eh
    from core.criterion import KLLoss, L1Loss, lsgan_adversarial_loss
    from utils.utils import FullModel_encdec
    cfg = make_cfg(True)
    torch.manual_seed(0)
    ed = eh.get_encdec_model(cfg)
    ez = eh.get_encz_model(cfg)
    ds = eh.get_D_sequence_model(cfg)
    df = eh.get_D_frame_model(cfg)
    fm = FullModel_encdec(ez, ed, ds, df, L1Loss(), KLLoss(), lsgan_adversarial_loss(),
                          1.0, 0.1, 1.0, gan)
    return fm, cfg


def _inputs(B=2, H=32, W=32, L=3):
    import torch
    g = torch.Generator().manual_seed(1)
    return [torch.randn(B, 3 * L, H, W, generator=g) for _ in range(3)]


def run_eval(tag="tiny_eval", B=2):
    """Eval-mode prior-sampling forward (function.py:60,124-136) on a trained-looking state."""
    import torch
    fm, cfg = _full_model(gan=1.0)
    zc = cfg.MODEL.EXTRA.Z_DIM
    gen = torch.Generator().manual_seed(7)
    sd = fm.state_dict()
    with torch.no_grad():
        for k in sorted(sd):
            v = sd[k]
            if not v.is_floating_point():
                continue
            stem = k.rsplit(".", 1)[0]
            is_bn = stem + ".running_mean" in sd
            if k.endswith("running_mean"):
                v.copy_(0.3 * torch.randn(v.shape, generator=gen))
            elif k.endswith("running_var"):
                v.copy_(0.5 + 1.5 * torch.rand(v.shape, generator=gen))
            elif v.dim() == 4:  # conv weight: variance-preserving scale
                v.copy_(torch.randn(v.shape, generator=gen) / float(v[0].numel()) ** 0.5)
            elif k.endswith(".weight") and is_bn:
                v.copy_(1.0 + 0.2 * torch.randn(v.shape, generator=gen))
            else:  # BN bias, conv bias
                v.copy_(0.1 * torch.randn(v.shape, generator=gen))
    fm.eval()
    xt, x2t, x3t = _inputs(B)
    torch.manual_seed(321)
    with torch.no_grad():
        losses, x1p, x2p, x3p = fm(xt, x2t, x3t, 1.0, sampling_mode="prior_sampling")
    torch.manual_seed(321)  # replay: z (prior) then the encoder's random code
    z = torch.randn(B, zc, 1, 1)
    code = torch.randn(B, zc, 1, 1)
    out = {"xt": xt, "x2t": x2t, "x3t": x3t, "eps": z, "code": code,
           "x1p": x1p, "x2p": x2p, "x3p": x3p}
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL", "gan_seq", "gan_frame"]
    for n, v in zip(names, losses):
        out["loss_" + n] = torch.as_tensor(float(v.reshape(-1)[0]) if torch.is_tensor(v) else v)
    for k, v in fm.state_dict().items():
        out["sd/" + k] = v
    arrays = {k: v.detach().numpy() for k, v in out.items()}
    path = os.path.join(HERE, f"{tag}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def run_ckpt(tag="ref_ckpt", B=2):
    """The reference's own checkpoint (train.py:320-324) after one ELBO step + Adam, and
    the next step taken from it."""
    import torch
    fm, cfg = _full_model(gan=0.0)
    zc = cfg.MODEL.EXTRA.Z_DIM
    fm.train()
    named = [(n, p) for n, p in fm.named_parameters() if p.requires_grad and "D_model" not in n]
    opt = torch.optim.Adam([{"params": [p for _, p in named]}], lr=1e-4)  # train.py:251-256
    xt, x2t, x3t = _inputs(B)
    torch.manual_seed(123)
    losses = fm(xt, x2t, x3t, 1.0)[0]
    opt.zero_grad()
    losses[0].backward()
    opt.step()
    ck = os.path.join(HERE, "ref_checkpoint_encdec.pth.tar")
    torch.save({"epoch": 1, "state_dict": fm.state_dict(),
                "optimizer_encdec": opt.state_dict()}, ck)
    print(f"wrote {ck} ({os.path.getsize(ck) / 1e6:.2f} MB)")
    torch.manual_seed(124)
    losses = fm(xt, x2t, x3t, 1.0)[0]
    torch.manual_seed(124)
    eps = torch.randn(B, zc, 1, 1)
    code = torch.randn(B, zc, 1, 1)
    out = {"xt": xt, "x2t": x2t, "x3t": x3t, "eps": eps, "code": code}
    names = ["loss_all", "xt_recon", "x2t_recon", "x3t_recon", "z_KL"]
    for n, v in zip(names, losses):
        out["loss_" + n] = torch.as_tensor(float(v.reshape(-1)[0]))
    opt.zero_grad()
    losses[0].backward()
    opt.step()
    pn, psum, pabs = checksums({n: p.detach() for n, p in named})
    out["param_sum"] = torch.as_tensor(psum)
    out["param_abs"] = torch.as_tensor(pabs)
    arrays = {k: v.detach().numpy() for k, v in out.items()}
    arrays["param_names"] = np.array(pn)
    path = os.path.join(HERE, f"{tag}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


EXTRA = {"tiny_eval": run_eval, "ref_ckpt": run_ckpt}


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    np.int = int  # the reference uses the removed numpy alias (enc_hrnet.py:321,596,700)
    import torch
    torch.set_num_threads(8)
    for tag in (sys.argv[1:] or list(CASES) + list(EXTRA)):
        if tag in EXTRA:
            EXTRA[tag]()
        else:
            run_case(tag, **CASES[tag])


if __name__ == "__main__":
    main()
