"""VAE² prior-sampling evaluation CLI on MI355X (drop-in for the reference's
tools/inference.py:57-201).

    python tools/inference.py --cfg experiments/vae2_w18_small_v2_128x256.yaml \
        TRAIN.RESUME True DATASET.TRAIN_SET <list of clip zips> [KEY VALUE ...]

Same flow: config -> logger -> models (encz skipped for DETERMINISTIC) -> clips with the
fixed window (random_pos=False) in list order -> FullModel_encdec -> the encdec
checkpoint of the training run when TRAIN.RESUME -> core.function.inference for epoch 0
under no_grad (MI355X.EVAL_SAMPLES prior samples per clip, 100 as the reference).
"""
import argparse
import os
import pprint
import sys

import torch

import _init_paths  # noqa: F401
import models  # noqa: F401
from config import config, update_config
from core.criterion import KLLoss, L1Loss, lsgan_adversarial_loss
from core.function import inference
from utils.utils import FullModel_encdec, create_logger

from train import build_loader
from vae2.trainer import NullWriter


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description="VAE2 inference (MI355X)")
    parser.add_argument("--cfg", help="experiment configure file name", required=True, type=str)
    parser.add_argument("--local_rank", "--local-rank", type=int,
                        default=int(os.environ.get("LOCAL_RANK", "0")))
    parser.add_argument("opts", help="Modify config options using the command-line", default=None,
                        nargs=argparse.REMAINDER)
    args = parser.parse_args(argv)
    update_config(config, args)
    return args


def main(argv=None):
    args = parse_args(argv)
    logger, final_output_dir, _ = create_logger(config, args.cfg, "train")
    logger.info(pprint.pformat(args))
    logger.info(config)
    device = torch.device("cuda:{}".format(args.local_rank))
    torch.cuda.set_device(device)
    extra = config.MODEL.EXTRA
    encdec_model = models.enc_hrnet.get_encdec_model(config)
    encz_model = (models.enc_hrnet.get_encz_model(config)
                  if extra.BASELINE_MODE != "DETERMINISTIC" else None)
    loader, _, n_clips = build_loader(config, config.DATASET.TRAIN_SET, False, device, logger,
                                      random_pos=False)
    model_encdec = FullModel_encdec(
        encz_model=encz_model, encdec_model=encdec_model, D_model_sequence=None,
        D_model_frame=None, criterion_recon=L1Loss(), criterion_KL=KLLoss(),
        criterion_gan=lsgan_adversarial_loss(), x1recon_lambda=config.TRAIN.X1RECON_LAMBDA,
        x2recon_lambda=config.TRAIN.X2RECON_LAMBDA, x3recon_lambda=config.TRAIN.X3RECON_LAMBDA,
        gan_lambda=config.TRAIN.GAN_LAMBDA).to(device)
    epoch_iters = int(n_clips / config.TRAIN.BATCH_SIZE_PER_GPU / max(1, len(config.GPUS)))
    if config.TRAIN.RESUME:  # inference.py:165-175
        state_file = os.path.join(final_output_dir, "checkpoint_encdec.pth.tar")
        if os.path.isfile(state_file):
            ck = torch.load(state_file, map_location="cpu", weights_only=True)
            # the training checkpoint may hold the discriminators' keys (GAN runs)
            sd = {k: v for k, v in ck["state_dict"].items() if not k.startswith("D_model")}
            model_encdec.load_state_dict(sd)
            logger.info("=> loaded checkpoint (epoch {})".format(ck["epoch"]))
    writer_dict = {"writer": NullWriter(), "train_global_steps": 0, "valid_global_steps": 0}
    return inference(config, 0, config.TRAIN.END_EPOCH, epoch_iters, config.TRAIN.LR,
                     config.TRAIN.END_EPOCH * epoch_iters, loader, None, None, model_encdec,
                     None, writer_dict, device, final_output_dir,
                     use_multiplier=config.TRAIN.USE_X2RECON_MULTIPLIER,
                     is_baseline=extra.IS_BASELINE, baseline_mode=extra.BASELINE_MODE)


if __name__ == "__main__":
    main()
    sys.exit(0)
