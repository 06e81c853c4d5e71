"""ELBO criteria with the reference's call signatures (criterion.py:61-103).

Tensors handed in by callers are NCHW (or any dense layout): L1 is a sum over
elements and does not depend on layout.  Inside FullModel_encdec the fused
NHWC paths of vae2.ops are used directly.
"""
import torch
import torch.nn as nn

from . import ops


class L1Loss(nn.Module):
    """sum |predict - target| / batch  (criterion.py:61-69)."""

    def forward(self, predict, target):
        return ops.l1(predict, target, 1.0 / predict.shape[0], flat=True)


def _muvar_nhwc(m, v):
    # (N, z, h, w) NCHW pair -> (N, h, w, 2z) NHWC
    return ops.to_nhwc(torch.cat([m, v], dim=1))


class KLLoss(nn.Module):
    """sum 0.5 (mu^2 + exp(logvar) - logvar - 1) / batch, list-aware (criterion.py:72-87)."""

    def forward(self, mu, logvar):
        if isinstance(mu, (list, tuple)):
            assert isinstance(logvar, (list, tuple))
            terms = [self._one(m, v) for m, v in zip(mu, logvar)]
            return ops.weighted_sum(terms, [1.0] * len(terms))
        return self._one(mu, logvar)

    @staticmethod
    def _one(m, v):
        mv = _muvar_nhwc(m, v)
        eps = torch.zeros(mv.shape[:3] + (mv.shape[3] // 2,), device=mv.device)
        _, kl = ops.reparam_kl(mv, eps, prior=False, scale=1.0 / m.shape[0])
        return kl


class lsgan_adversarial_loss(nn.Module):  # noqa: N801 (reference name)
    """sum (sample - 1)^2 / batch for 'real', sum sample^2 / batch for 'fake'
    (MSELoss(reduction='sum') against ones / zeros, criterion.py:90-103)."""

    def forward(self, sample, mode):
        assert mode in ["real", "fake"]
        return ops.lsgan(sample, mode == "real", 1.0 / sample.shape[0], flat=True)
