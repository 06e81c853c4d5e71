"""VAE² training CLI on MI355X (drop-in for the reference's tools/train.py).

    python tools/train.py --cfg experiments/vae2_w18_small_v2_128x256.yaml [KEY VALUE ...]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/train.py --cfg ... GPUS "(0,1,2,3,4,5,6,7)"

Flow (reference train.py:55-353): parse args + YAML -> logger -> models (same
factories, same RNG order) -> process group (RCCL) -> dataset / sampler / loader
-> FullModel_encdec -> SyncBN statistics + flat-gradient all-reduce (instead of
DDP) -> Adam -> resume -> epoch loop -> rank-0 checkpoints with the reference's
file and key names.

Deliberate differences: `TRAIN.OPTIMIZER: sgd` raises a clear ValueError (the
reference crashes with a TypeError on `p.name`, train.py:234); single-GPU
checkpoints are written (the reference calls `.module` on a non-DDP model,
train.py:322); epochs past END_EPOCH use the main loader when no
DATASET.EXTRA_TRAIN_SET is given (the reference raises a NameError there);
`MI355X.ELBO_ONLY True` drops the two discriminators (the ELBO step alone; the
reference always builds them and runs the D step); the Cityscapes sequence zips are
decoded once into a uint8 cache and normalised on the GPU (MI355X.CLIP_CACHE, default),
or replaced by MI355X.SYNTHETIC_DATA clips when that switch is set; the dataset is given
TRAIN.CLIP_LENGTH (the reference leaves CityscapesSequence at its default 3).
"""
import argparse
import os
import pprint
import shutil
import sys
import timeit

import torch

import _init_paths  # noqa: F401
import datasets  # noqa: F401  (lib/datasets: the drop-in CityscapesSequence)
import models  # noqa: F401
from config import config, update_config
from core.criterion import KLLoss, L1Loss, lsgan_adversarial_loss
from core.function import adversarial_train
from utils.utils import FullModel_D, FullModel_encdec, create_logger

from vae2 import clips
from vae2 import dist as vdist
from vae2.optim import FusedAdam
from vae2.trainer import NullWriter, SyntheticClips


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description="Train VAE2 (MI355X)")
    parser.add_argument("--cfg", help="experiment configure file name", required=True, type=str)
    parser.add_argument("--local_rank", "--local-rank", type=int,
                        default=int(os.environ.get("LOCAL_RANK", "0")))
    parser.add_argument("opts", help="Modify config options using the command-line", default=None,
                        nargs=argparse.REMAINDER)
    args = parser.parse_args(argv)
    update_config(config, args)
    return args


def build_loader(cfg, list_path, shuffle, device, logger=None, random_pos=True):
    """(loader, number of clips) for one list file (train.py:113-140).

    MI355X.SYNTHETIC_DATA: Gaussian clips.  Otherwise the Cityscapes sequence zips
    (DATASET.ROOT + a list file, gen_cityscapes_data.py layout): with MI355X.CLIP_CACHE
    decoded once into a uint8 cache (rank 0 builds it, the others wait) and served by
    ClipLoader (pinned staging + HIP normalisation); without it the drop-in
    CityscapesSequence through a torch DataLoader (PIL decode per item, uint8 windows
    normalised on the GPU by adversarial_train)."""
    w, h = cfg.TRAIN.IMAGE_SIZE
    B = cfg.TRAIN.BATCH_SIZE_PER_GPU
    if cfg.MI355X.SYNTHETIC_DATA:
        dataset = SyntheticClips(cfg.MI355X.SYNTHETIC_CLIPS, cfg.TRAIN.CLIP_LENGTH, h, w)
    elif cfg.DATASET.DATASET != "cityscapessequence":
        raise ValueError("VAE2 trains on DATASET.DATASET cityscapessequence (got {})"
                         .format(cfg.DATASET.DATASET))
    elif cfg.MI355X.CLIP_CACHE:
        cdir = cfg.MI355X.CLIP_CACHE_DIR or clips.cache_dir_for(cfg.DATASET.ROOT, list_path,
                                                                (h, w))
        if vdist.rank() == 0:
            clips.build_cache(cfg.DATASET.ROOT, list_path, (h, w), cache_dir=cdir,
                              log=logger.info if logger else None)
        if vdist.is_dist():
            torch.distributed.barrier()
        cache = clips.ClipCache(cdir)
        sampler = (torch.utils.data.distributed.DistributedSampler(range(len(cache)))
                   if vdist.is_dist() else None)
        loader = clips.ClipLoader(cache, B, clip_length=cfg.TRAIN.CLIP_LENGTH, clip_num=3,
                                  sampler=sampler, shuffle=shuffle and sampler is None,
                                  random_pos=random_pos, device=device)
        return loader, sampler, len(cache)
    else:
        dataset = datasets.cityscapessequence(
            root=cfg.DATASET.ROOT, list_path=list_path, num_samples=None,
            num_classes=cfg.DATASET.NUM_CLASSES, multi_scale=cfg.TRAIN.MULTI_SCALE,
            flip=cfg.TRAIN.FLIP, ignore_label=cfg.TRAIN.IGNORE_LABEL,
            base_size=cfg.TRAIN.BASE_SIZE, crop_size=(h, w),
            downsample_rate=cfg.TRAIN.DOWNSAMPLERATE, scale_factor=cfg.TRAIN.SCALE_FACTOR,
            clip_length=cfg.TRAIN.CLIP_LENGTH, random_pos=random_pos,
            fixed_length=cfg.DATASET.FIXED_LENGTH)
    sampler = torch.utils.data.distributed.DistributedSampler(dataset) if vdist.is_dist() else None
    loader = torch.utils.data.DataLoader(
        dataset, batch_size=B, shuffle=shuffle and sampler is None, num_workers=cfg.WORKERS,
        pin_memory=True, drop_last=True, sampler=sampler)
    return loader, sampler, len(dataset)


def main(argv=None):
    args = parse_args(argv)
    logger, final_output_dir, tb_log_dir = create_logger(config, args.cfg, "train")
    logger.info(pprint.pformat(args))
    logger.info(config)
    writer_dict = {"writer": NullWriter(), "train_global_steps": 0, "valid_global_steps": 0}
    try:
        from tensorboardX import SummaryWriter
        writer_dict["writer"] = SummaryWriter(tb_log_dir)
    except ImportError:
        logger.info("tensorboardX not installed: scalars are logged to the text log only")

    gpus = list(config.GPUS)
    distributed = len(gpus) > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1
    if config.TRAIN.OPTIMIZER != "adam":
        raise ValueError("Only Support ADAM optimizer (the reference's sgd path is broken)")
    extra = config.MODEL.EXTRA

    # models, in the reference's construction order (train.py:79-82)
    encdec_model = models.enc_hrnet.get_encdec_model(config)
    encz_model = (models.enc_hrnet.get_encz_model(config)
                  if extra.BASELINE_MODE != "DETERMINISTIC" else None)
    use_d = not config.MI355X.ELBO_ONLY
    D_model_sequence = models.enc_hrnet.get_D_sequence_model(config) if use_d else None
    D_model_frame = models.enc_hrnet.get_D_frame_model(config) if use_d else None

    if args.local_rank == 0:
        this_dir = os.path.dirname(os.path.abspath(__file__))
        dst = os.path.join(final_output_dir, "models")
        if os.path.exists(dst):
            shutil.rmtree(dst)
        shutil.copytree(os.path.join(this_dir, "..", "lib", "models"), dst)

    if distributed:
        vdist.init("nccl")
        vdist.set_sync_bn(config.MI355X.SYNC_BN)
        if config.MI355X.SYNC_BN and config.MI355X.SYNC_BN_EXCHANGE == "ipc":
            vdist.init_syncbn_ipc()
    device = torch.device("cuda:{}".format(args.local_rank))
    torch.cuda.set_device(device)

    loader, sampler, n_clips = build_loader(config, config.DATASET.TRAIN_SET,
                                            config.TRAIN.SHUFFLE, device, logger)
    extra_loader, extra_sampler = loader, sampler
    if config.DATASET.EXTRA_TRAIN_SET:  # train.py:142-167
        extra_loader, extra_sampler, _ = build_loader(config, config.DATASET.EXTRA_TRAIN_SET,
                                                      config.TRAIN.SHUFFLE, device, logger)

    model_encdec = FullModel_encdec(
        encz_model=encz_model, encdec_model=encdec_model, D_model_sequence=D_model_sequence,
        D_model_frame=D_model_frame, criterion_recon=L1Loss(), criterion_KL=KLLoss(),
        criterion_gan=lsgan_adversarial_loss(), x1recon_lambda=config.TRAIN.X1RECON_LAMBDA,
        x2recon_lambda=config.TRAIN.X2RECON_LAMBDA, x3recon_lambda=config.TRAIN.X3RECON_LAMBDA,
        gan_lambda=config.TRAIN.GAN_LAMBDA)
    model_encdec.defer_checks = config.MI355X.DEFER_CHECKS
    model_encdec = model_encdec.to(device)
    model_D = None
    if use_d:
        model_D = FullModel_D(D_model_sequence=D_model_sequence, D_model_frame=D_model_frame,
                              criterion_gan=lsgan_adversarial_loss()).to(device)
        assert model_encdec.D_model_sequence is model_D.D_model_sequence, "Unexpected behavior."
        assert model_encdec.D_model_frame is model_D.D_model_frame, "Unexpected behavior."
    # Adam over encz + ED ('D_model' excluded) and over the discriminators (train.py:251-261)
    nets = [m for m in (encz_model, encdec_model) if m is not None]
    optimizer = FusedAdam(nets, lr=config.TRAIN.LR)
    optimizer_D = FusedAdam([D_model_sequence, D_model_frame], lr=config.TRAIN.LR) if use_d \
        else None
    if vdist.is_dist():  # replicas start identical (DDP's initial broadcast)
        for opt in (optimizer, optimizer_D):
            for f in (opt.flats if opt is not None else []):
                torch.distributed.broadcast(f.data, src=0)

    epoch_iters = int(n_clips / config.TRAIN.BATCH_SIZE_PER_GPU / max(1, len(gpus)))
    last_epoch = 0
    state_file = os.path.join(final_output_dir, "checkpoint_encdec.pth.tar")
    state_file_D = os.path.join(final_output_dir, "checkpoint_D.pth.tar")
    if config.TRAIN.RESUME:  # train.py:270-290
        if os.path.isfile(state_file):
            ck = torch.load(state_file, map_location="cpu", weights_only=True)
            last_epoch = ck["epoch"]
            model_encdec.load_state_dict(ck["state_dict"], strict=use_d)
            optimizer.load_state_dict(ck["optimizer_encdec"])
            logger.info("=> loaded checkpoint (epoch {})".format(ck["epoch"]))
        if use_d and os.path.isfile(state_file_D):
            ck = torch.load(state_file_D, map_location="cpu", weights_only=True)
            last_epoch = ck["epoch"]
            model_D.load_state_dict(ck["state_dict"])
            optimizer_D.load_state_dict(ck["optimizer_D"])
            logger.info("=> loaded checkpoint (epoch {})".format(ck["epoch"]))

    start = timeit.default_timer()
    end_epoch = config.TRAIN.END_EPOCH + config.TRAIN.EXTRA_EPOCH
    num_iters = config.TRAIN.END_EPOCH * epoch_iters
    extra_iters = config.TRAIN.EXTRA_EPOCH * epoch_iters
    for epoch in range(last_epoch, end_epoch):
        if sampler is not None:
            sampler.set_epoch(epoch)
        if extra_sampler is not None and extra_sampler is not sampler:
            extra_sampler.set_epoch(epoch)
        if epoch >= config.TRAIN.END_EPOCH:  # train.py:300-306
            # EXTRA_LR reaches adversarial_train as base_lr, which only logs it: the
            # reference's adjust_learning_rate call is commented out (function.py:525-528),
            # so the optimizers keep training at TRAIN.LR in the extra epochs too
            ep_args = (epoch - config.TRAIN.END_EPOCH, config.TRAIN.EXTRA_EPOCH, epoch_iters,
                       config.TRAIN.EXTRA_LR, extra_iters, extra_loader)
        else:
            ep_args = (epoch, config.TRAIN.END_EPOCH, epoch_iters, config.TRAIN.LR, num_iters,
                       loader)
        adversarial_train(config, *ep_args, optimizer, optimizer_D, model_encdec, model_D,
                          writer_dict, device, final_output_dir,
                          use_multiplier=config.TRAIN.USE_X2RECON_MULTIPLIER,
                          is_baseline=extra.IS_BASELINE, baseline_mode=extra.BASELINE_MODE)
        if vdist.rank() == 0:  # train.py:317-348
            logger.info("=> saving checkpoint to {}".format(state_file))
            torch.save({"epoch": epoch + 1, "state_dict": model_encdec.state_dict(),
                        "optimizer_encdec": optimizer.state_dict()}, state_file)
            if use_d:
                logger.info("=> saving checkpoint to {}".format(state_file_D))
                torch.save({"epoch": epoch + 1, "state_dict": model_D.state_dict(),
                            "optimizer_D": optimizer_D.state_dict()}, state_file_D)
            if epoch == end_epoch - 1:
                torch.save(model_encdec.state_dict(),
                           os.path.join(final_output_dir, "model_encdec_final_state.pth"))
                if use_d:
                    torch.save(model_D.state_dict(),
                               os.path.join(final_output_dir, "model_D_final_state.pth"))
                writer_dict["writer"].close()
                logger.info("Hours: %d" % int((timeit.default_timer() - start) / 3600))
                logger.info("Done")
        if vdist.is_dist():
            # the other ranks wait here for rank 0's checkpoint writes: otherwise they would
            # start the next epoch and wait in its first SyncBN exchange, whose bounded wait
            # can expire during a slow save
            torch.distributed.barrier()


if __name__ == "__main__":
    sys.exit(main())
