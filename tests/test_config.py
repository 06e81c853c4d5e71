"""yacs-compatible config surface (reference lib/config/default.py:121-127)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
YAML = os.path.join(ROOT, "vae-2_amd", "experiments", "vae2_w18_small_v2_128x256.yaml")


def fresh():
    sys.path.insert(0, os.path.join(ROOT, "vae-2_amd", "lib"))
    from config.default import _C
    return _C.clone()


def test_yaml_and_cli_merge():
    cfg = fresh()

    class A:
        cfg = YAML
        opts = ["TRAIN.BATCH_SIZE_PER_GPU", "4", "GPUS", "(0,1)", "TRAIN.LR", "0.001"]

    from config.default import update_config
    update_config(cfg, A)
    assert cfg.is_frozen()
    assert cfg.TRAIN.IMAGE_SIZE == [256, 128]
    assert cfg.TRAIN.BATCH_SIZE_PER_GPU == 4
    assert cfg.GPUS == (0, 1)
    assert cfg.TRAIN.LR == 0.001
    assert cfg.MODEL.EXTRA.Z_DIM == 10
    assert cfg.MODEL.EXTRA["STAGE4"]["NUM_CHANNELS"] == [18, 36, 72, 144]
    assert cfg.MODEL.EXTRA.STAGE2.BLOCK == "BASIC"
    with pytest.raises(AttributeError):
        cfg.TRAIN.LR = 1.0


def test_unknown_keys_and_type_errors():
    cfg = fresh()
    with pytest.raises(KeyError):
        cfg.merge_from_list(["TRAIN.NOT_A_KEY", "1"])
    with pytest.raises(ValueError):
        cfg.merge_from_list(["TRAIN.BATCH_SIZE_PER_GPU", "'eight'"])
    cfg.merge_from_list(["MODEL.EXTRA.NEW_KEY", "3"])  # EXTRA has new_allowed (default.py:38)
    assert cfg.MODEL.EXTRA.NEW_KEY == 3
    cfg.merge_from_list(["TRAIN.LR", "1"])  # int accepted for a float key
    assert isinstance(cfg.TRAIN.LR, float)
