"""Evaluation metrics on the GPU (vae2.metrics over vae2_to_image / vae2_ssim /
vae2_avgpool2x2 / vae2_absdiff_sqdiff_sum) against oracle/metrics_ref.py.

_to_image is the reference's own arithmetic (function.py:86-97): bit-exact.  recon_loss
and PSNR (function.py:252, criterion.py:106-116): double sums, 1e-6 relative.  SSIM /
MS-SSIM restate pytorch_msssim 1.0.0, which is absent here (parity unpinned by
reference outputs): fp32 kernels vs the float64 restatement, 2e-5 absolute."""
import numpy as np
import pytest
import torch

from oracle import metrics_ref

pytestmark = pytest.mark.gpu


def _frames(shape, seed, noise=0.3):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(shape, generator=g)
    b = a + noise * torch.randn(shape, generator=g)
    return a, b


def test_to_image_bit_exact():
    from vae2 import metrics
    a, _ = _frames((2, 9, 20, 36), 0, 0)
    a[0, 0, 0, :4] = torch.tensor([-5.0, 5.0, 0.0, -2.1179])  # clipped both ways
    got = metrics.to_image(a.cuda()).cpu().numpy()
    for n in range(2):
        for f in range(3):
            ref = metrics_ref.to_image(a[n, 3 * f:3 * f + 3].numpy())
            assert np.array_equal(got[n, 3 * f:3 * f + 3].transpose(1, 2, 0), ref)


@pytest.mark.parametrize("hw", [(11, 11), (32, 64), (77, 131), (128, 256)])
def test_ssim_matches_restatement(hw):
    from vae2 import metrics
    a, b = _frames((2, 3) + hw, sum(hw))
    a = metrics.to_image(a.cuda())
    b = metrics.to_image(b.cuda())
    got = metrics.ssim_planes(a, b).cpu().numpy()
    s, cs = metrics_ref._ssim(a.cpu().numpy(), b.cpu().numpy(), 255, metrics_ref.gauss_win())
    assert np.abs(got[..., 0] - s).max() < 2e-5
    assert np.abs(got[..., 1] - cs).max() < 2e-5
    v = float(metrics.ssim(a, b, data_range=255, size_average=True))
    assert abs(v - s.mean()) < 2e-5
    # identical images: SSIM 1
    one = metrics.ssim_planes(a, a).cpu().numpy()
    assert np.abs(one - 1).max() < 1e-5


@pytest.mark.parametrize("hw", [(7, 9), (8, 8), (33, 64), (161, 175)])
def test_avg_pool2_matches_restatement(hw):
    from vae2 import metrics
    a, _ = _frames((1, 3) + hw, 3, 0)
    got = metrics.avg_pool2(a.cuda()).cpu().numpy()
    ref = metrics_ref._avg_pool2(a.numpy().astype(np.float64))
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-6


@pytest.mark.parametrize("hw", [(176, 176), (256, 512), (173, 197)])
def test_ms_ssim_matches_restatement(hw):
    from vae2 import metrics
    a, b = _frames((1, 3) + hw, 9)
    a = metrics.to_image(a.cuda())
    b = metrics.to_image(b.cuda())
    w = [1.0 / 3.0] * 3
    got = float(metrics.ms_ssim(a, b, data_range=255, weights=w))
    ref = metrics_ref.ms_ssim(a.cpu().numpy(), b.cpu().numpy(), 255, w)
    assert abs(got - ref) < 2e-5
    got5 = float(metrics.ms_ssim(a, b, data_range=255))
    ref5 = metrics_ref.ms_ssim(a.cpu().numpy(), b.cpu().numpy(), 255,
                               [0.0448, 0.2856, 0.3001, 0.2363, 0.1333])
    assert abs(got5 - ref5) < 2e-5


def test_ms_ssim_size_assertion_and_shape_errors():
    from vae2 import metrics
    a = torch.rand(1, 3, 128, 256, device="cuda") * 255
    with pytest.raises(AssertionError):
        metrics.ms_ssim(a, a)
    with pytest.raises(ValueError):
        metrics.ssim(a, a[:, :, :64])


def test_recon_psnr_and_frame_metrics():
    from vae2 import metrics
    p, t = _frames((6, 40, 48), 21)
    res, ai, bi = metrics.frame_metrics(p.cuda(), t.cuda())
    for f in range(2):
        im = metrics_ref.to_image(p[3 * f:3 * f + 3].numpy())
        gt = metrics_ref.to_image(t[3 * f:3 * f + 3].numpy())
        assert abs(res[f, 0] - metrics_ref.recon_loss(im, gt)) < 1e-6 * max(1, res[f, 0])
        assert abs(res[f, 3] - metrics_ref.psnr(im, gt)) < 1e-6 * res[f, 3]
        X = im.transpose(2, 0, 1)[None]
        Y = gt.transpose(2, 0, 1)[None]
        assert abs(res[f, 1] - metrics_ref.ssim(X, Y)) < 2e-5
        assert np.isnan(res[f, 2])  # 40x48 is below pytorch_msssim's MS-SSIM size bound
    psnr = float(metrics.PSNR()(ai[0], bi[0]))
    assert abs(psnr - res[0, 3]) < 1e-4


def test_psnr_and_recon_match_reference_fixture():
    """recon_loss and PSNR of the GPU metric path against the reference's own PSNR class
    (tests/golden/metrics.npz, made by tests/golden/make_golden_metrics.py)."""
    import os
    from helpers import GOLDEN
    from vae2 import metrics
    g = np.load(os.path.join(GOLDEN, "metrics.npz"))
    for k in range(3):
        a = metrics.to_image(torch.from_numpy(g[f"{k}/a"])[None].cuda())
        b = metrics.to_image(torch.from_numpy(g[f"{k}/b"])[None].cuda())
        psnr = float(metrics.PSNR()(a, b))
        s = metrics.absdiff_sqdiff(a, b).cpu()
        recon = float(s[0]) / a.numel()
        assert abs(psnr - float(g[f"{k}/psnr"])) <= 1e-5 * abs(float(g[f"{k}/psnr"]))
        assert abs(recon - float(g[f"{k}/recon"])) <= 1e-5 * abs(float(g[f"{k}/recon"]))
        if min(a.shape[-2:]) >= 11:  # the SSIM kernels need the 11-tap window to fit
            res, _, _ = metrics.frame_metrics(torch.from_numpy(g[f"{k}/a"]).cuda(),
                                              torch.from_numpy(g[f"{k}/b"]).cuda())
            assert abs(res[0, 3] - float(g[f"{k}/psnr"])) <= 1e-5 * abs(float(g[f"{k}/psnr"]))
