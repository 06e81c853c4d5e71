# Drop-in for the reference's lib/models package (only the VAE² model module).
from . import enc_hrnet  # noqa: F401
