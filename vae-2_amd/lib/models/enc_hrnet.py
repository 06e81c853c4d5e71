"""Drop-in for reference lib/models/enc_hrnet.py: HRNet VAE² nets on the HIP path."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from vae2.hrnet import (BLOCKS as blocks_dict, BN_MOMENTUM, BasicBlock, Bottleneck,  # noqa: E402,F401
                        HighResolutionModule, HighResolutionNet, HighResolutionNetDsc,
                        HighResolutionNetED, HighResolutionNetEDz, get_D_frame_model,
                        get_D_sequence_model, get_encdec_model, get_encz_model)
