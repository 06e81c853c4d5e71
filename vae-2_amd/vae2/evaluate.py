"""Prior-sampling evaluation (reference lib/core/function.py:55-316, tools/inference.py).

For every clip batch: NUM_SAMPLES forward passes of the eval-mode model with
sampling_mode='prior_sampling' (z ~ N(0, I)); rank 0 then writes, for the LAST clip of the
batch (the reference only looks at index -1), the ground-truth frames as PNGs and, per
sample and predicted frame, recon (mean |a - b|), SSIM, MS-SSIM (weights [1/3]*3) and
PSNR of the [0, 255] images into the reference's text files, plus a PNG whose name
carries the metrics:

  <out>/vis/epoch<e>/<name>/x1t_<i>.png, x2t_<i>.png, x3t_<i>.png
  <out>/vis/epoch<e>/<name>/x2tpredict/x2t_<i>_{recon,ssim,msssim,psnr}loss.txt
  <out>/vis/epoch<e>/<name>/x2tpredict/x2t_<i>_trial_<s>_recon.._ssim.._msssim...png
  (x3tpredict/ likewise; in baseline mode x2t_hat is scored against x3t, :242)

The forward passes and every metric run on the GPU (vae2.metrics); only the scalars and
the uint8 frames come back to the host.  Deliberate differences: MS-SSIM is written as
nan when a frame is below pytorch_msssim's size bound (min side <= 160), where the
reference's call would raise; the 10-D toy example's plots ('toyexample' names, a
CUDA-only MLP outside the HRNet path) are not supported.
"""
import os

import numpy as np
import torch

from . import clips
from . import metrics
from .trainer import dynamic_coeff, get_rank


def _png(img_f32_hwc, path):
    from PIL import Image
    Image.fromarray(img_f32_hwc.astype(np.uint8)).save(path)


def _f32str(v):
    """str() of the reference's values: recon is a numpy float32, ssim / msssim / psnr are
    .item() of float32 tensors."""
    return str(np.float32(v))


def _item(v):
    return str(float(np.float32(v)))


def inference(config, epoch, num_epoch, epoch_iters, base_lr, num_iters, trainloader,
              optimizer_encdec, optimizer_D, model_encdec, model_D, writer_dict, device,
              final_output_dir, use_multiplier, is_baseline=False, baseline_mode=None,
              seeds=None, num_samples=None):
    model_encdec.eval()
    rank = get_rank()
    multiplier = dynamic_coeff(max_iters=num_epoch, cur_iters=epoch) if use_multiplier else 1.0
    if num_samples is None:
        num_samples = getattr(getattr(config, "MI355X", None), "EVAL_SAMPLES", 100)
    results = []
    with torch.no_grad():
        for i_iter, batch in enumerate(trainloader):
            xs, name = batch
            if "toyexample" in name[-1]:
                raise NotImplementedError("the 10-D toy example is outside the HRNet path")
            if torch.is_tensor(xs) or len(xs) == 3:
                xt, x2t, x3t = clips.batch_to_device(xs, device)
                xt_last = x3t_last = None
            else:  # momentum-sampling 5-segment clips (function.py:109-115)
                assert len(xs) == 5
                xs = [x.to(device) for x in xs]
                xt_last, x3t_last, xt, x2t, x3t = xs[0], xs[2], xs[2], xs[3], xs[4]
            cand = []
            for s in range(num_samples):
                _, xt_p, x2t_p, x3t_p = model_encdec(
                    xt=xt, x2t=x2t, x3t=x3t, multiplier=multiplier,
                    sampling_mode="prior_sampling", xt_last=xt_last, x3t_last=x3t_last,
                    is_baseline=is_baseline, baseline_mode=baseline_mode)
                cand.append((x2t_p[-1].clone(), x3t_p[-1].clone()))
            if rank != 0:
                continue
            save = os.path.join(final_output_dir, "vis", "epoch{}".format(epoch), name[-1])
            os.makedirs(save, exist_ok=True)
            for tag, x in (("x1t", xt), ("x2t", x2t), ("x3t", x3t)):
                F = x.shape[1] // 3
                im = metrics.to_image(x[-1].reshape(F, 3, *x.shape[2:])).cpu().numpy()
                for i in range(F):
                    _png(im[i].transpose(1, 2, 0), os.path.join(save, f"{tag}_{i}.png"))
            per_clip = {}
            for tag, k, gt in (("x2t", 0, x3t if is_baseline else x2t), ("x3t", 1, x3t)):
                d = os.path.join(final_output_dir, "vis", "epoch{}".format(epoch), name[-1],
                                 f"{tag}predict")
                os.makedirs(d, exist_ok=True)
                rows = []
                for s in range(num_samples):
                    m, a, _ = metrics.frame_metrics(cand[s][k], gt[-1])
                    a = a.cpu().numpy()
                    rows.append(m)
                    for i in range(m.shape[0]):
                        recon, ss, ms, ps = m[i]
                        for suffix, val in (("reconloss", _f32str(recon)),
                                            ("ssimloss", _item(ss)),
                                            ("msssimloss", _item(ms)),
                                            ("psnrloss", _item(ps))):
                            with open(os.path.join(d, f"{tag}_{i}_{suffix}.txt"), "a") as fw:
                                fw.write(val + "\n")
                        _png(a[i].transpose(1, 2, 0), os.path.join(
                            d, "{}_{}_trial_{}_recon{}_ssim{}_msssim{}.png".format(
                                tag, i, s, _f32str(recon), _item(ss), _item(ms))))
                per_clip[tag] = np.stack(rows)  # [samples][frames][recon, ssim, msssim, psnr]
            results.append((name[-1], per_clip))
    return results
