"""Evaluation metrics of the prior-sampling inference on the HIP path.

  to_image        function.py:86-97 (x*std + mean, *255, clip)   -> vae2_to_image
  recon / PSNR    function.py:252, criterion.py:106-116          -> vae2_absdiff_sqdiff_sum
  ssim, ms_ssim   pytorch_msssim 1.0.0 (function.py:24-25, :244-251; third-party, absent
                  from the reference tree and from this image: restated, see
                  oracle/metrics_ref.py)                          -> vae2_ssim, vae2_avgpool2x2

Images are CUDA fp32 NCHW tensors; a frame is 3 planes.  The kernels return per-plane
(or per-tensor) sums / means in double; the last combination (the per-level product of
MS-SSIM over a handful of per-plane numbers, log10 of PSNR) is host arithmetic on those.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .ops import ptr, stream_ptr

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)

_WINS = {}


def _win(device, size, sigma):
    """pytorch_msssim _fspecial_gauss_1d (fp32): exp(-(i - size//2)^2 / (2 sigma^2)),
    normalised."""
    key = (str(device), size, float(sigma))
    w = _WINS.get(key)
    if w is None:
        coords = torch.arange(size, dtype=torch.float32) - size // 2
        g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
        g /= g.sum()
        w = g.to(device)
        _WINS[key] = w
    return w


def _check(X, Y):
    if X.shape != Y.shape:
        raise ValueError(f"Input images should have the same dimensions, but got {X.shape} "
                         f"and {Y.shape}.")
    if X.dim() != 4:
        raise ValueError(f"Input images should be 4-d tensors, but got {X.shape}")
    if X.dtype != torch.float32 or Y.dtype != torch.float32 or not (X.is_cuda and Y.is_cuda):
        raise ValueError("metrics take CUDA float32 tensors")
    return X.contiguous(), Y.contiguous()


def to_image(x, mean=MEAN, std=STD, out=None):
    """[N][C][H][W] normalised frames (C a multiple of 3) -> [0, 255] float images, same
    layout (the reference's _to_image before its HWC transpose / uint8 cast)."""
    x = x.contiguous()
    N, C, H, W = x.shape
    y = torch.empty_like(x) if out is None else out
    m = (ctypes.c_double * 3)(*mean)
    s = (ctypes.c_double * 3)(*std)
    _lib.call("vae2_to_image", ptr(x), ptr(y), N, C, H, W, m, s, stream_ptr())
    return y


def _ws(planes, h, w, device):
    n = _lib.load().vae2_metrics_ws_size(planes, h, w)
    return torch.empty(n, dtype=torch.float64, device=device)


def absdiff_sqdiff(a, b):
    """(sum |a-b|, sum (a-b)^2) as a CUDA float64 tensor [2]."""
    a, b = a.contiguous(), b.contiguous()
    if a.shape != b.shape:
        raise ValueError("shape mismatch")
    out = torch.empty(2, dtype=torch.float64, device=a.device)
    _lib.call("vae2_absdiff_sqdiff_sum", ptr(a), ptr(b), a.numel(),
              ptr(_ws(1, 1, 1, a.device)), ptr(out), stream_ptr())
    return out


def ssim_planes(X, Y, data_range=255, win_size=11, win_sigma=1.5, K=(0.01, 0.03)):
    """Per-(n, c) mean SSIM and CS maps: CUDA float64 [N][C][2]."""
    X, Y = _check(X, Y)
    N, C, H, W = X.shape
    out = torch.empty((N, C, 2), dtype=torch.float64, device=X.device)
    c1 = (K[0] * data_range) ** 2
    c2 = (K[1] * data_range) ** 2
    _lib.call("vae2_ssim", ptr(X), ptr(Y), N * C, H, W, ptr(_win(X.device, win_size, win_sigma)),
              win_size, c1, c2, ptr(_ws(N * C, H, W, X.device)), ptr(out), stream_ptr())
    return out


def avg_pool2(x):
    x = x.contiguous()
    N, C, H, W = x.shape
    ph, pw = H % 2, W % 2
    y = torch.empty((N, C, (H + 2 * ph - 2) // 2 + 1, (W + 2 * pw - 2) // 2 + 1),
                    dtype=x.dtype, device=x.device)
    _lib.call("vae2_avgpool2x2", ptr(x), ptr(y), N * C, H, W, stream_ptr())
    return y


def ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5,
         K=(0.01, 0.03), nonnegative_ssim=False):
    """pytorch_msssim.ssim: mean over channels (and batch if size_average)."""
    if not win_size % 2 == 1:
        raise ValueError("Window size should be odd.")
    v = ssim_planes(X, Y, data_range, win_size, win_sigma, K)[..., 0]
    if nonnegative_ssim:
        v = v.clamp_min(0)
    return (v.mean() if size_average else v.mean(1)).float()


def ms_ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5,
            weights=None, K=(0.01, 0.03)):
    """pytorch_msssim.ms_ssim (the reference binds weights=[1/3]*3, function.py:25)."""
    X, Y = _check(X, Y)
    if not win_size % 2 == 1:
        raise ValueError("Window size should be odd.")
    smaller_side = min(X.shape[-2:])
    assert smaller_side > (win_size - 1) * (2 ** 4), \
        "Image size should be larger than %d due to the 4 downsamplings in ms-ssim" % (
            (win_size - 1) * (2 ** 4))
    if weights is None:
        weights = [0.0448, 0.2856, 0.3001, 0.2363, 0.1333]
    w = torch.as_tensor(weights, dtype=torch.float32).double().cpu().numpy()
    levels = len(w)
    vals = []
    for i in range(levels):
        v = ssim_planes(X, Y, data_range, win_size, win_sigma, K)
        if i < levels - 1:
            vals.append(v[..., 1])
            X, Y = avg_pool2(X), avg_pool2(Y)
    vals.append(v[..., 0])
    arr = torch.stack(vals, 0).cpu().numpy()  # [levels][N][C]
    ms = np.prod(np.maximum(arr, 0) ** w[:, None, None], axis=0)
    return torch.tensor(ms.mean() if size_average else ms.mean(1), dtype=torch.float32)


class PSNR:
    """criterion.py:106-116: 20 log10(255 / sqrt(mean (img1 - img2)^2))."""

    def __init__(self):
        self.name = "PSNR"

    @staticmethod
    def __call__(img1, img2):
        s = absdiff_sqdiff(img1, img2).cpu()
        mse = float(s[1]) / img1.numel()
        return torch.tensor(20 * np.log10(255.0 / np.sqrt(mse)), dtype=torch.float32)


def frame_metrics(pred, gt, mean=MEAN, std=STD, msssim_weights=(1.0 / 3.0,) * 3):
    """Per frame of one sample's clip tensors pred, gt ([3F][H][W], normalised): the
    reference's (recon_loss, ssim, ms_ssim, psnr) of the [0, 255] images
    (function.py:240-261) -> float64 numpy [F][4]; ms_ssim is NaN when the frame is too
    small for pytorch_msssim's size assertion (the reference would raise there)."""
    F3, H, W = pred.shape
    F = F3 // 3
    a = to_image(pred.reshape(F, 3, H, W), mean, std)
    b = to_image(gt.reshape(F, 3, H, W), mean, std)
    sp = ssim_planes(a, b)  # [F][3][2]
    sums = torch.stack([absdiff_sqdiff(a[f], b[f]) for f in range(F)], 0)  # [F][2]
    ok = min(H, W) > 10 * 16
    ms = [float(ms_ssim(a[f:f + 1], b[f:f + 1], weights=list(msssim_weights)))
          if ok else float("nan") for f in range(F)]
    sp = sp.cpu().numpy()
    sums = sums.cpu().numpy()
    n = 3 * H * W
    out = np.empty((F, 4))
    out[:, 0] = sums[:, 0] / n
    out[:, 1] = sp[:, :, 0].mean(1)
    out[:, 2] = ms
    with np.errstate(divide="ignore"):
        out[:, 3] = 20 * np.log10(255.0 / np.sqrt(sums[:, 1] / n))
    return out, a, b
