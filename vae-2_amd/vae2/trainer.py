"""Training-loop pieces of the ELBO path.

  adversarial_train   per-epoch loop (function.py:443-553): H2D, ELBO forward,
                      loss reduce, zero_grad / backward / RCCL grad all-reduce /
                      Adam, the discriminator step (FullModel_D, Adam on the D
                      parameters), meters, PRINT_FREQ logging.
  SyntheticClips      Cityscapes-shaped clips (3 segments x CLIP_LENGTH RGB frames
                      stacked on channels, cityscapes.py:311-326) for
                      benchmarking and CI; the zip/PNG clips are vae2/clips.py.
  create_logger, AverageMeter, get_world_size, get_rank   (utils.py)
"""
import logging
import math
import os
import time
from pathlib import Path

import torch

from . import clips
from . import dist as vdist


class AverageMeter:
    def __init__(self):
        self.initialized = False
        self.val = self.avg = self.sum = self.count = None

    def initialize(self, val, weight):
        self.val, self.avg, self.sum, self.count = val, val, val * weight, weight
        self.initialized = True

    def update(self, val, weight=1):
        if not self.initialized:
            self.initialize(val, weight)
        else:
            self.val = val
            self.sum += val * weight
            self.count += weight
            self.avg = self.sum / self.count

    def value(self):
        return self.val

    def average(self):
        return self.avg


def get_world_size():
    return vdist.world_size()


def get_rank():
    return vdist.rank()


def dynamic_coeff(max_iters, cur_iters):
    """KL annealing multiplier (utils.py:465-468)."""
    return math.sin((math.pi / 2) * (float(cur_iters) / float(max_iters)))


def create_logger(cfg, cfg_name, phase="train"):
    """output/<dataset>/<cfg name>/ + log/<...>/ + a file+console logger (utils.py:400-432)."""
    root_output_dir = Path(cfg.OUTPUT_DIR)
    root_output_dir.mkdir(parents=True, exist_ok=True)
    dataset = cfg.DATASET.DATASET
    model = cfg.MODEL.NAME
    cfg_name = os.path.basename(cfg_name).split(".")[0]
    final_output_dir = root_output_dir / dataset / cfg_name
    final_output_dir.mkdir(parents=True, exist_ok=True)
    time_str = time.strftime("%Y-%m-%d-%H-%M")
    log_file = "{}_{}_{}.log".format(cfg_name, time_str, phase)
    logging.basicConfig(filename=str(final_output_dir / log_file),
                        format="%(asctime)-15s %(message)s")
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    logging.getLogger("").addHandler(logging.StreamHandler())
    tb_log_dir = Path(cfg.LOG_DIR) / dataset / model / (cfg_name + "_" + time_str)
    tb_log_dir.mkdir(parents=True, exist_ok=True)
    return logger, str(final_output_dir), str(tb_log_dir)


class SyntheticClips(torch.utils.data.Dataset):
    """Deterministic Gaussian clips shaped like CityscapesSequence items:
    ([xt, x2t, x3t], name), each (3*clip_length, H, W) fp32."""

    def __init__(self, num_clips, clip_length, height, width, seed=1):
        self.n, self.L, self.h, self.w, self.seed = num_clips, clip_length, height, width, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        x = torch.randn(3, 3 * self.L, self.h, self.w, generator=g)
        return [x[0], x[1], x[2]], "synthetic_{:06d}".format(i)


class NullWriter:
    def add_scalar(self, *a, **k):
        pass

    def close(self):
        pass


def adversarial_train(config, epoch, num_epoch, epoch_iters, base_lr, num_iters, trainloader,
                      optimizer_encdec, optimizer_D, model_encdec, model_D, writer_dict, device,
                      final_output_dir, use_multiplier, is_baseline=False, baseline_mode=None,
                      seeds=None):
    """One epoch of the VAE² ELBO step (function.py:443-553)."""
    model_encdec.train()
    if model_D is not None:
        model_D.train()
    fm = getattr(model_encdec, "module", model_encdec)
    batch_time = AverageMeter()
    ave_loss_D = AverageMeter()
    ave_loss_encdec = AverageMeter()
    tic = time.time()
    writer = writer_dict["writer"]
    global_steps = writer_dict["train_global_steps"]
    rank = get_rank()
    world_size = get_world_size()
    multiplier = dynamic_coeff(max_iters=num_epoch, cur_iters=epoch) if use_multiplier else 1.0
    flats = optimizer_encdec.flats
    for i_iter, batch in enumerate(trainloader):
        xs, name = batch
        xt, x2t, x3t = clips.batch_to_device(xs, device)  # uint8 windows: HIP normalisation
        losses, xt_predict, x2t_predict, x3t_predict = model_encdec(
            xt=xt, x2t=x2t, x3t=x3t, multiplier=multiplier, is_baseline=is_baseline,
            baseline_mode=baseline_mode)
        (loss_encdec, loss_xt_recon, loss_x2t_recon, loss_x3t_recon, loss_z_KL,
         loss_x2t_gan_sequence, loss_x2t_gan_frame) = losses
        reduced_loss_encdec = vdist.reduce_tensor(loss_encdec.detach().clone())
        optimizer_encdec.zero_grad()
        loss_encdec.backward()
        vdist.allreduce_grads(flats)
        optimizer_encdec.step()
        if model_D is not None and (not is_baseline or baseline_mode == "VAE_GAN"):
            # D step (function.py:503-512): real x2t (x3t in baseline) vs detached x2t_hat
            losses_D = model_D(x2t=x2t if not is_baseline else x3t,
                               x2t_predict=x2t_predict.detach())
            loss_D, loss_D_sequence, loss_D_frame = losses_D
            reduced_loss_D = vdist.reduce_tensor(loss_D.detach().clone())
            optimizer_D.zero_grad()
            loss_D.backward()
            vdist.allreduce_grads(optimizer_D.flats)
            optimizer_D.step()
        else:
            reduced_loss_D = torch.zeros(1)
            loss_D_sequence = loss_D_frame = 0.0
        if i_iter % config.PRINT_FREQ == 0:
            if getattr(fm, "defer_checks", False):
                fm.check_anomalies()  # deferred NaN/Inf flag (utils.py:63-65), one sync
            vdist.syncbn_check()  # a timed-out IPC SyncBN exchange raises here
        batch_time.update(time.time() - tic)
        tic = time.time()
        ave_loss_D.update(float(reduced_loss_D.item()))
        ave_loss_encdec.update(float(reduced_loss_encdec.item()))
        if i_iter % config.PRINT_FREQ == 0 and rank == 0:
            print_loss_D = ave_loss_D.average() / world_size
            print_loss_encdec = ave_loss_encdec.average() / world_size
            f = lambda t: float(t) if not torch.is_tensor(t) else float(t.item())  # noqa: E731
            msg = ("Epoch: [{}/{}] Iter:[{}/{}], Time: {:.2f}, lr: {:.6f}, Loss_D_ave: {:.6f}, "
                   "Loss_D_sequence: {:.6f}, Loss_D_frame: {:.6f}, Loss_encdec_ave: {:.6f},"
                   "loss_xt_recon: {:.6f}, loss_x2t_recon: {:.6f}, loss_x3t_recon: {:.6f}，"
                   "loss_z_KL: {:.6f}, loss_x2t_gan_sequence: {:.6f}, loss_x2t_gan_frame: {:.6f}"
                   ).format(epoch, num_epoch, i_iter, epoch_iters, batch_time.average(), base_lr,
                            print_loss_D, f(loss_D_sequence), f(loss_D_frame), print_loss_encdec,
                            f(loss_xt_recon), f(loss_x2t_recon), f(loss_x3t_recon), f(loss_z_KL),
                            f(loss_x2t_gan_sequence), f(loss_x2t_gan_frame))
            logging.info(msg)
            for tag, val in (("train_loss_D", print_loss_D),
                             ("train_loss_D_sequence", f(loss_D_sequence)),
                             ("train_loss_D_frame", f(loss_D_frame)),
                             ("train_loss_encdec", print_loss_encdec),
                             ("train_loss_xt_recon", f(loss_xt_recon)),
                             ("train_loss_x2_recon", f(loss_x2t_recon)),
                             ("train_loss_x3t_recon", f(loss_x3t_recon)),
                             ("train_loss_z_KL", f(loss_z_KL)),
                             ("train_loss_x2t_gan_sequence", f(loss_x2t_gan_sequence)),
                             ("train_loss_x2t_gan_frame", f(loss_x2t_gan_frame))):
                writer.add_scalar(tag, val, global_steps)
            writer_dict["train_global_steps"] = global_steps + 1
    vdist.syncbn_check()  # once per epoch as well (the last iterations after a PRINT_FREQ point)
