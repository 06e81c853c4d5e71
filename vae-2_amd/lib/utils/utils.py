"""Drop-in for reference lib/utils/utils.py: the ELBO wrapper and training helpers."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from vae2.model import FullModel_D, FullModel_encdec  # noqa: E402,F401
from vae2.trainer import (AverageMeter, create_logger, dynamic_coeff,  # noqa: E402,F401
                          get_rank, get_world_size)
