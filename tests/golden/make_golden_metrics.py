"""Generate tests/golden/metrics.npz: the reference's own PSNR (lib/core/criterion.py:106-116)
on [0, 255] image pairs built with the reference's _to_image arithmetic
(function.py:86-97, restated in oracle/metrics_ref.py: the function is nested inside
inference() and cannot be imported).  Runs ONLY in the build container; imports
/root/reference/lib/core/criterion.py read-only and writes data only.

SSIM / MS-SSIM come from pytorch_msssim, which is neither in /root/reference nor
installed here: no reference fixture exists for them (parity unpinned, see
oracle/metrics_ref.py).

    python tests/golden/make_golden_metrics.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/lib"


def main():
    sys.path.insert(0, REF)
    sys.path.insert(0, REPO)
    from core.criterion import PSNR  # the reference's class
    from oracle.metrics_ref import to_image
    psnr = PSNR()
    rng = np.random.RandomState(21)
    out = {}
    for k, (h, w, noise) in enumerate([(16, 32, 0.3), (40, 48, 0.05), (7, 9, 1.0)]):
        a = rng.randn(3, h, w).astype(np.float32)
        b = (a + noise * rng.randn(3, h, w)).astype(np.float32)
        ia, ib = to_image(a), to_image(b)  # [H][W][3] float32 in [0, 255]
        out[f"{k}/a"] = a
        out[f"{k}/b"] = b
        out[f"{k}/psnr"] = np.float32(psnr(torch.from_numpy(ia), torch.from_numpy(ib)).item())
        out[f"{k}/recon"] = np.float32(np.mean(np.abs(ia - ib)))  # function.py:252
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), **out)
    print("wrote", os.path.join(HERE, "metrics.npz"), sorted(out))


if __name__ == "__main__":
    main()
