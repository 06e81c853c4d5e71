# Drop-in for the reference's lib/config (config/__init__.py): same names.
from .default import _C as config  # noqa: F401
from .default import update_config  # noqa: F401
from .models import MODEL_EXTRAS  # noqa: F401
