"""Drop-in for reference lib/utils/utils.py: the ELBO wrapper and training helpers."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from vae2.model import FullModel_encdec  # noqa: E402,F401
from vae2.trainer import (AverageMeter, create_logger, dynamic_coeff,  # noqa: E402,F401
                          get_rank, get_world_size)


class FullModel_D:  # noqa: N801 (reference name)
    """Discriminator wrapper (utils.py:244-276): GAN path, SURVEY.md §8f next-1."""

    def __init__(self, *a, **k):
        raise NotImplementedError("the GAN discriminator step is not implemented yet")
