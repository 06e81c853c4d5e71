# Drop-in for the reference's lib/datasets package: the VAE² clip dataset
# (tools/train.py:115 evaluates 'datasets.' + DATASET.DATASET).
from .cityscapes import CityscapesSequence as cityscapessequence  # noqa: F401
from .cityscapes import CityscapesSequence  # noqa: F401
