"""Drop-in for reference lib/core/function.py: the ELBO training loop and the
prior-sampling evaluation."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from vae2.dist import reduce_tensor  # noqa: E402,F401
from vae2.trainer import adversarial_train  # noqa: E402,F401
from vae2.evaluate import inference  # noqa: E402,F401
