"""Config schema read by the VAE² training path (reference lib/config/default.py:17-127).

Same keys and defaults as the reference so its YAMLs and `KEY VALUE` CLI
overrides apply unchanged, plus an `MI355X` node for build-only switches.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from vae2.config import CfgNode  # noqa: E402

_SCHEMA = {
    "OUTPUT_DIR": "", "LOG_DIR": "", "GPUS": (0,), "WORKERS": 4, "PRINT_FREQ": 20,
    "AUTO_RESUME": False, "PIN_MEMORY": True, "RANK": 0,
    "CUDNN": {"BENCHMARK": True, "DETERMINISTIC": False, "ENABLED": True},
    "MODEL": {"NAME": "enc_hrnet", "PRETRAINED": ""},
    "LOSS": {"USE_OHEM": False, "OHEMTHRES": 0.9, "OHEMKEEP": 100000, "CLASS_BALANCE": True},
    "DATASET": {
        "ROOT": "/data/yizhou/cityscape/leftImg8bit_sequence_resized_zip/",
        "DATASET": "cityscapes", "NUM_CLASSES": 19,
        "TRAIN_SET": "/data/yizhou/cityscape/trainval_list.text", "EXTRA_TRAIN_SET": "",
        "TEST_SET": "/data/yizhou/cityscape/test_list.text", "FIXED_LENGTH": False,
    },
    "TRAIN": {
        "IMAGE_SIZE": [512, 256], "BASE_SIZE": 512, "DOWNSAMPLERATE": 1, "FLIP": False,
        "MULTI_SCALE": False, "SCALE_FACTOR": 16, "CLIP_LENGTH": 3,
        "X1RECON_LAMBDA": 1.0, "X2RECON_LAMBDA": 0.1, "X3RECON_LAMBDA": 1.0, "GAN_LAMBDA": 1.0,
        "USE_X2RECON_MULTIPLIER": False, "LR_FACTOR": 0.1, "LR_STEP": [90, 110], "LR": 0.01,
        "EXTRA_LR": 0.001, "OPTIMIZER": "sgd", "MOMENTUM": 0.9, "WD": 0.0001, "NESTEROV": False,
        "IGNORE_LABEL": -1, "BEGIN_EPOCH": 0, "END_EPOCH": 484, "EXTRA_EPOCH": 0,
        "RESUME": False, "BATCH_SIZE_PER_GPU": 32, "SHUFFLE": True, "NUM_SAMPLES": 0,
    },
    "TEST": {
        "IMAGE_SIZE": [512, 256], "BASE_SIZE": 512, "BATCH_SIZE_PER_GPU": 32, "NUM_SAMPLES": 0,
        "MODEL_FILE": "", "FLIP_TEST": False, "MULTI_SCALE": False, "CENTER_CROP_TEST": False,
        "SCALE_LIST": [1],
    },
    "DEBUG": {"DEBUG": False, "SAVE_BATCH_IMAGES_GT": False, "SAVE_BATCH_IMAGES_PRED": False,
              "SAVE_HEATMAPS_GT": False, "SAVE_HEATMAPS_PRED": False},
    # build-only switches (not in the reference)
    "MI355X": {
        "SYNC_BN": True,          # global BN statistics when distributed (reference: SyncBatchNorm)
        # SyncBN statistics exchange: "ipc" = the one-shot peer all-reduce kernel
        # (vae2_syncbn_allreduce, node-local, self-checked at start; RCCL if it does not come
        # up), "rccl" = torch.distributed all_reduce
        "SYNC_BN_EXCHANGE": "ipc",
        "HIP_GRAPH": False,       # capture the training step in a hipGraph
        "DEFER_CHECKS": False,    # one NaN/Inf host read per step instead of four
        "SYNTHETIC_DATA": False,  # Cityscapes-shaped Gaussian clips instead of the zip dataset
        "SYNTHETIC_CLIPS": 64,
        "ELBO_ONLY": False,       # no discriminators / D step (the ELBO step alone)
        "CLIP_CACHE": True,       # zip clips: decode once to a uint8 cache, GPU normalisation
        "CLIP_CACHE_DIR": "",     # default <DATASET.ROOT>/.vae2_cache/<list>_<H>x<W>
        "EVAL_SAMPLES": 100,      # prior samples per clip in tools/inference.py (function.py:124)
    },
}

_C = CfgNode(_SCHEMA)
_C.MODEL.EXTRA = CfgNode({"IS_BASELINE": False, "BASELINE_MODE": "VAE_NATIVE"}, new_allowed=True)


def update_config(cfg, args):
    cfg.defrost()
    cfg.merge_from_file(args.cfg)
    cfg.merge_from_list(args.opts)
    cfg.freeze()
