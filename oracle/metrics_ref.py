"""ORACLE — test infrastructure only, never on the product path.

float64 numpy restatement of the evaluation metrics of the prior-sampling inference
(function.py:55-316, tools/inference.py), the checker of vae2/metrics.py:

  _to_image        function.py:86-97       x*std + mean, *255, clip [0, 255] (float32
                                           array against float64 mean/std, as numpy does)
  recon_loss       function.py:252         mean |a - b|
  PSNR             criterion.py:106-116    20 log10(255 / sqrt(mean (a - b)^2))
  ssim / ms_ssim   pytorch_msssim (function.py:24-25, called at :244-251 with
                   data_range=255, MS-SSIM weights [1/3]*3)

pytorch_msssim is a third-party dependency that is NOT in /root/reference and is not
installed here (requirements.txt:14, unpinned).  Restated from its published 1.0.0
algorithm: 1-D Gaussian window (win_size 11, sigma 1.5, normalised), applied separably
as a valid convolution along H then W; C1 = (0.01 L)^2, C2 = (0.03 L)^2;
cs_map = (2 s12 + C2) / (s1 + s2 + C2), ssim_map = (2 mu1 mu2 + C1) / (mu1^2 + mu2^2 + C1)
* cs_map; per-channel means; ms_ssim: per level relu(cs), avg_pool2d(2, padding = size
% 2) between levels, relu(ssim) at the last level, prod(level values ** weights), mean;
it asserts min(H, W) > (win_size - 1) * 2**4.  SSIM / MS-SSIM parity is therefore
UNPINNED by reference outputs (no fixture of the dependency exists offline); _to_image,
recon_loss and PSNR are restated from the reference's own code.
"""
import numpy as np


def to_image(x, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """x: float32 [3][H][W] -> float32 [H][W][3] in [0, 255] (function.py:86-97)."""
    x = np.transpose(np.asarray(x, dtype=np.float32), (1, 2, 0)).copy()
    x *= np.asarray([std], dtype=np.float64)
    x += np.asarray([mean], dtype=np.float64)
    x *= 255.0
    np.clip(x, 0, 255, out=x)
    return x


def recon_loss(a, b):
    return float(np.mean(np.abs(a.astype(np.float64) - b.astype(np.float64))))


def psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return float(20 * np.log10(255.0 / np.sqrt(mse)))


def gauss_win(size=11, sigma=1.5):
    coords = np.arange(size, dtype=np.float32) - size // 2
    g = np.exp(-(coords ** 2) / np.float32(2 * sigma ** 2)).astype(np.float32)
    return (g / g.sum()).astype(np.float32)


def _filter(x, win):
    """valid separable filtering of [..., H, W] along H then W (float64)."""
    k = len(win)
    w = win.astype(np.float64)
    H, W = x.shape[-2:]
    y = sum(w[i] * x[..., i:H - k + 1 + i, :] for i in range(k))
    return sum(w[i] * y[..., :, i:W - k + 1 + i] for i in range(k))


def _ssim(X, Y, data_range, win, K=(0.01, 0.03)):
    """per-(n, c) mean SSIM and CS maps of [N][C][H][W] images."""
    X = X.astype(np.float64)
    Y = Y.astype(np.float64)
    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    mu1, mu2 = _filter(X, win), _filter(Y, win)
    s1 = _filter(X * X, win) - mu1 ** 2
    s2 = _filter(Y * Y, win) - mu2 ** 2
    s12 = _filter(X * Y, win) - mu1 * mu2
    cs_map = (2 * s12 + C2) / (s1 + s2 + C2)
    ssim_map = ((2 * mu1 * mu2 + C1) / (mu1 ** 2 + mu2 ** 2 + C1)) * cs_map
    return ssim_map.mean(axis=(-2, -1)), cs_map.mean(axis=(-2, -1))


def ssim(X, Y, data_range=255, win_size=11, win_sigma=1.5):
    return float(_ssim(X, Y, data_range, gauss_win(win_size, win_sigma))[0].mean())


def _avg_pool2(x):
    H, W = x.shape[-2:]
    ph, pw = H % 2, W % 2
    xp = np.pad(x, [(0, 0)] * (x.ndim - 2) + [(ph, ph), (pw, pw)])
    Ho, Wo = (H + 2 * ph - 2) // 2 + 1, (W + 2 * pw - 2) // 2 + 1
    xp = xp[..., :2 * Ho, :2 * Wo]
    return 0.25 * (xp[..., 0::2, 0::2] + xp[..., 1::2, 0::2] + xp[..., 0::2, 1::2]
                   + xp[..., 1::2, 1::2])


def ms_ssim(X, Y, data_range=255, weights=(1 / 3, 1 / 3, 1 / 3), win_size=11, win_sigma=1.5):
    assert min(X.shape[-2:]) > (win_size - 1) * 2 ** 4
    win = gauss_win(win_size, win_sigma)
    w = np.asarray(weights, dtype=np.float32).astype(np.float64)
    mcs = []
    X = X.astype(np.float64)
    Y = Y.astype(np.float64)
    for i in range(len(w)):
        s, cs = _ssim(X, Y, data_range, win)
        if i < len(w) - 1:
            mcs.append(np.maximum(cs, 0))
            X, Y = _avg_pool2(X), _avg_pool2(Y)
    vals = np.stack(mcs + [np.maximum(s, 0)], 0)
    return float(np.prod(vals ** w[:, None, None], axis=0).mean())
