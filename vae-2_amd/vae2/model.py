"""FullModel_encdec: the VAE² ELBO step (utils.py:39-155) on the HIP path.

Same constructor and forward signature / return structure as the reference:
    forward(xt, x2t, x3t, multiplier, is_baseline=False, baseline_mode='VAE_NATIVE',
            sampling_mode='default', xt_last=None, x3t_last=None)
    -> ([loss_all (1,), xt_recon, x2t_recon, x3t_recon, z_KL, gan_seq, gan_frame],
        xt_hat, x2t_hat, x3t_hat)                       (all NCHW, like the reference)

Inside, clips are converted once to NHWC; the posterior net, sampler, the
encoder / two decoders and the L1 / KL terms all run on libvae2_hip kernels.

Noise: eps and the encoder's random code are drawn from PyTorch's default CPU
generator in the reference's order (eps first, then the code)
and copied to the device, so a seeded run reproduces the reference's CPU draws.
`set_noise(eps, code)` injects them explicitly (tests, benchmarks).

Anomaly checks (utils.py:63-65) keep the reference's AssertionError semantics;
they are evaluated on a device flag, and `defer_checks=True` postpones the host
read to `check_anomalies()` (one sync instead of four per step).

GAN terms (utils.py:114-119): with discriminators attached they are formed as the
reference does (always in non-baseline mode, for VAE_GAN in baseline mode).  The
reference backpropagates the generator loss into the discriminators too, and the
D step then zeroes those gradients (function.py:499-510); here the discriminator
parameters are frozen during the generator pass so no weight gradient is computed
for them (same results, less work).  With GAN_LAMBDA 0 the terms are evaluated
without autograd (their gradient is exactly zero).

FullModel_D (utils.py:244-276): the discriminator loss of the D step.
"""
import contextlib

import torch
import torch.nn as nn

from . import ops, streams

_MODES = ("VAE_NATIVE", "VAE_ANNEAL", "VAE_GAN", "DETERMINISTIC")


class FullModel_encdec(nn.Module):  # noqa: N801 (reference name)
    def __init__(self, encz_model, encdec_model, D_model_sequence, D_model_frame,
                 criterion_recon, criterion_KL, criterion_gan,
                 x1recon_lambda=1.0, x2recon_lambda=1.0, x3recon_lambda=1.0, gan_lambda=1.0):
        super().__init__()
        self.encz_model = encz_model
        self.encdec_model = encdec_model
        self.D_model_sequence = D_model_sequence
        self.D_model_frame = D_model_frame
        self.criterion_recon = criterion_recon
        self.criterion_KL = criterion_KL
        self.criterion_gan = criterion_gan
        self.x1recon_lambda = x1recon_lambda
        self.x2recon_lambda = x2recon_lambda
        self.x3recon_lambda = x3recon_lambda
        self.gan_lambda = gan_lambda
        self.defer_checks = False
        self._flag = None
        self._noise = None

    # ---- noise / checks -------------------------------------------------------
    def set_noise(self, eps=None, code=None):
        """Use these draws for the next forward (NCHW; eps may be a list with HD_Z)."""
        self._noise = (eps, code)

    def _draw(self, shapes_eps, code_shape, device, prior):
        if self._noise is not None:
            eps, code = self._noise
            self._noise = None
        else:
            if isinstance(shapes_eps, list):
                eps = [torch.randn(*s) for s in shapes_eps]
            else:
                eps = torch.randn(*shapes_eps) if shapes_eps is not None else None
            code = torch.randn(*code_shape) if code_shape is not None else None
        return eps, code

    def _check(self, named):
        for name, t in named:
            tensors = t if isinstance(t, (list, tuple)) else [t]
            self._flag = ops.nonfinite_flag(tensors, self._flag)
            if not self.defer_checks:
                bad = int(self._flag.item())
                self._flag.zero_()
                assert not bad, "{} got nan or inf".format(name)

    def check_anomalies(self):
        """Host-read the deferred NaN/Inf flag (raises AssertionError like the reference)."""
        streams.join_all()
        if self._flag is not None:
            bad = int(self._flag.item())
            self._flag.zero_()
            assert not bad, "step got nan or inf"

    def _gan_terms(self, x2p, nframes):
        """0.5*LSGAN(D_seq(x2t_hat), real), sum_f 0.5*LSGAN(D_frame(frame f), real)."""
        ds, df = self.D_model_sequence, self.D_model_frame
        if ds is None or df is None:
            return 0.0, 0.0
        B = x2p.shape[0]
        grad = self.gan_lambda != 0 and torch.is_grad_enabled()
        with frozen([ds, df]) if grad else torch.no_grad():
            seq = ops.lsgan(ds.run(x2p), True, 0.5 / B)
            fl = [ops.lsgan(df.run(f), True, 0.5 / B)
                  for f in ops.split_frames(x2p, nframes)]
            frame = ops.weighted_sum(fl, [1.0] * len(fl))
        return seq, frame

    # ---- forward ---------------------------------------------------------------
    def forward(self, xt, x2t, x3t, multiplier, is_baseline=False, baseline_mode="VAE_NATIVE",
                sampling_mode="default", xt_last=None, x3t_last=None):
        assert sampling_mode in ["default", "prior_sampling", "momentum_sampling"]
        if sampling_mode == "momentum_sampling":
            assert xt_last is not None
            assert x3t_last is not None
        if baseline_mode not in _MODES:
            raise NotImplementedError("Not implemented Baseline Mode: {}".format(baseline_mode))
        B = xt.shape[0]
        dev = xt.device
        kl_lambda = self.x3recon_lambda * multiplier if baseline_mode == "VAE_ANNEAL" \
            else self.x3recon_lambda
        prior = sampling_mode == "prior_sampling"
        ed = self.encdec_model
        zc = ed.z_dim

        xt_n = ops.to_nhwc(xt)
        x2t_n = ops.to_nhwc(x2t)
        x3t_n = ops.to_nhwc(x3t)
        H, W = xt_n.shape[1:3]

        enc_in = ops.cat([xt_n, x2t_n], (H, W)) if is_baseline else xt_n
        z = None
        kl = None
        trunk = None
        if baseline_mode != "DETERMINISTIC":
            zin = [xt_n, x2t_n, x3t_n] if is_baseline else [xt_n, x3t_n]
            # posterior net + sampler on a side stream, concurrent with the encoder
            # trunk (stem .. stage 3 do not depend on z)
            with streams.on_side(0, inputs=zin) as sz:
                muvars = self.encz_model.run(ops.cat(zin, (H, W)))
                hd = isinstance(muvars, list)
                eps_shapes = ([(B, zc, m.shape[1], m.shape[2]) for m in muvars] if hd
                              else (B, zc, 1, 1))
                code_shape = (B, zc, 1, 1) if ed.enable_random_code else None
                eps, code = self._draw(eps_shapes, code_shape, dev, prior)
                mvs = muvars if hd else [muvars]
                epss = eps if hd else [eps]
                zs, kls = [], []
                for mv, e in zip(mvs, epss):
                    e_n = e.to(dev, non_blocking=True).permute(0, 2, 3, 1).contiguous()
                    zb, klb = ops.reparam_kl(mv, e_n, prior=prior, scale=1.0 / B)
                    zs.append(zb)
                    kls.append(klb)
                z = zs if hd else zs[0]
                kl = kls[0] if len(kls) == 1 else ops.weighted_sum(kls, [1.0] * len(kls))
            trunk = ed.encode_trunk(enc_in)
            streams.join(sz, [zs, kl, muvars])
            if not prior:
                self._check([("0", z)] if not hd else list(zip(map(str, range(len(zs))), zs)))
        else:
            code = None
            if ed.enable_random_code:
                _, code = self._draw(None, (B, zc, 1, 1), dev, prior)
        code_n = (code.to(dev, non_blocking=True).permute(0, 2, 3, 1).contiguous()
                  if code is not None else None)

        x1p, x2p, x3p = ed.run(enc_in, z, code_n, is_baseline, trunk)
        self._check([("xt_predict", x1p), ("x2t_predict", x2p), ("x3t_predict", x3p)])

        terms, lams = [], []
        scale = 1.0 / B
        if not is_baseline:
            xt_recon = ops.l1(x1p, xt_n, scale)
            x2t_recon = ops.l1(x2p, x2t_n, scale)
            x3t_recon = ops.l1(x3p, x3t_n, scale)
            z_kl = kl
            gan_seq, gan_frame = self._gan_terms(x2p, x2t.shape[1] // ed.clip_length)
            terms = [xt_recon, x2t_recon, x3t_recon, z_kl]
            lams = [self.x1recon_lambda, self.x2recon_lambda, self.x3recon_lambda, kl_lambda]
            if torch.is_tensor(gan_seq) and self.gan_lambda != 0:
                terms += [gan_seq, gan_frame]
                lams += [self.gan_lambda, self.gan_lambda]
        else:
            xt_recon = 0.0
            x3t_recon = 0.0
            x2t_recon = ops.l1(x2p, x3t_n, scale)
            terms, lams = [x2t_recon], [self.x2recon_lambda]
            gan_seq, gan_frame = 0.0, 0.0
            if baseline_mode in ("VAE_NATIVE", "VAE_ANNEAL"):
                z_kl = kl
                terms.append(z_kl)
                lams.append(kl_lambda)
            elif baseline_mode == "DETERMINISTIC":
                z_kl = 0.0
            else:  # VAE_GAN
                z_kl = kl
                terms.append(z_kl)
                lams.append(kl_lambda)
                gan_seq, gan_frame = self._gan_terms(x2p, x2t.shape[1] // ed.clip_length)
                if torch.is_tensor(gan_seq) and self.gan_lambda != 0:
                    terms += [gan_seq, gan_frame]
                    lams += [self.gan_lambda, self.gan_lambda]
        loss_all = ops.weighted_sum(terms, lams)
        preds = (ops.to_nchw(x1p), ops.to_nchw(x2p), ops.to_nchw(x3p))
        return ([torch.unsqueeze(loss_all, 0), xt_recon, x2t_recon, x3t_recon, z_kl, gan_seq,
                 gan_frame], *preds)


@contextlib.contextmanager
def frozen(modules):
    """Temporarily stop autograd from asking for these modules' parameter gradients."""
    params = [p for m in modules for p in m.parameters() if p.requires_grad]
    for p in params:
        p.requires_grad_(False)
    try:
        yield
    finally:
        for p in params:
            p.requires_grad_(True)


class FullModel_D(nn.Module):  # noqa: N801 (reference name)
    """Discriminator loss of the D step (utils.py:244-276):
        D_seq   = 0.5 LSGAN(D_seq(x2t), real) + 0.5 LSGAN(D_seq(x2t_hat), fake)
        D_frame = sum_f 0.5 LSGAN(D_frame(x2t_f), real) + 0.5 LSGAN(D_frame(x2t_hat_f), fake)
        D_all   = gan_lambda (D_seq + D_frame)
    Calls run in the reference's order (BatchNorm running statistics are updated per
    call).  Returns [D_all (1,), D_seq, D_frame]."""

    def __init__(self, D_model_sequence, D_model_frame, criterion_gan, gan_lambda=1.0):
        super().__init__()
        self.D_model_sequence = D_model_sequence
        self.D_model_frame = D_model_frame
        self.criterion_gan = criterion_gan
        self.gan_lambda = gan_lambda

    def forward(self, x2t, x2t_predict):
        ds, df = self.D_model_sequence, self.D_model_frame
        B = x2t.shape[0]
        nframes = x2t.shape[1] // ds.clip_length
        real = ops.to_nhwc(x2t.detach())
        fake = ops.to_nhwc(x2t_predict.detach())
        seq = ops.weighted_sum([ops.lsgan(ds.run(real), True, 0.5 / B),
                                ops.lsgan(ds.run(fake), False, 0.5 / B)], [1.0, 1.0])
        fr, ff = [], []
        for r, f in zip(ops.split_frames(real, nframes), ops.split_frames(fake, nframes)):
            fr.append(ops.lsgan(df.run(r), True, 0.5 / B))
            ff.append(ops.lsgan(df.run(f), False, 0.5 / B))
        frame = ops.weighted_sum([ops.weighted_sum(fr, [1.0] * len(fr)),
                                  ops.weighted_sum(ff, [1.0] * len(ff))], [1.0, 1.0])
        d_all = ops.weighted_sum([seq, frame], [self.gan_lambda, self.gan_lambda])
        return [torch.unsqueeze(d_all, 0), seq, frame]
