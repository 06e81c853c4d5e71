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
"""
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

    def _gan_terms(self):
        if self.gan_lambda != 0 and self.D_model_sequence is not None:
            raise NotImplementedError(
                "GAN terms need the discriminator path (SURVEY.md §8f next-1), not implemented "
                "yet: set TRAIN.GAN_LAMBDA 0 (ELBO step) or pass D models as None")
        return 0.0, 0.0

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
            gan_seq, gan_frame = self._gan_terms()
            terms = [xt_recon, x2t_recon, x3t_recon, z_kl]
            lams = [self.x1recon_lambda, self.x2recon_lambda, self.x3recon_lambda, kl_lambda]
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
                gan_seq, gan_frame = self._gan_terms()
        loss_all = ops.weighted_sum(terms, lams)
        preds = (ops.to_nchw(x1p), ops.to_nchw(x2p), ops.to_nchw(x3p))
        return ([torch.unsqueeze(loss_all, 0), xt_recon, x2t_recon, x3t_recon, z_kl, gan_seq,
                 gan_frame], *preds)
