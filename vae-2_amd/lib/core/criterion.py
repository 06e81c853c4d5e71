"""Drop-in for reference lib/core/criterion.py (ELBO criteria on the HIP path)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from vae2.criterion import KLLoss, L1Loss, lsgan_adversarial_loss  # noqa: E402,F401
from vae2.metrics import PSNR  # noqa: E402,F401
