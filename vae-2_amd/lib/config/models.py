"""MODEL_EXTRAS (reference lib/config/models.py): HRNet-W18-small-v2 extras used by
the VAE² YAML (experiments/vae2_w18_small_v2_128x256.yaml)."""
from .default import CfgNode

_W18_SMALL_V2 = CfgNode({
    "FINAL_CONV_KERNEL": 1,
    "STAGE1": {"NUM_MODULES": 1, "NUM_BRANCHES": 1, "BLOCK": "BOTTLENECK", "NUM_BLOCKS": [2],
               "NUM_CHANNELS": [64], "FUSE_METHOD": "SUM"},
    "STAGE2": {"NUM_MODULES": 1, "NUM_BRANCHES": 2, "BLOCK": "BASIC", "NUM_BLOCKS": [2, 2],
               "NUM_CHANNELS": [18, 36], "FUSE_METHOD": "SUM"},
    "STAGE3": {"NUM_MODULES": 3, "NUM_BRANCHES": 3, "BLOCK": "BASIC", "NUM_BLOCKS": [2, 2, 2],
               "NUM_CHANNELS": [18, 36, 72], "FUSE_METHOD": "SUM"},
    "STAGE4": {"NUM_MODULES": 2, "NUM_BRANCHES": 4, "BLOCK": "BASIC",
               "NUM_BLOCKS": [2, 2, 2, 2], "NUM_CHANNELS": [18, 36, 72, 144],
               "FUSE_METHOD": "SUM"},
})

MODEL_EXTRAS = {"enc_hrnet": _W18_SMALL_V2, "seg_hrnet": _W18_SMALL_V2}
