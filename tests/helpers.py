"""Shared test helpers: configs, model construction, golden fixtures."""
import copy
import os

import numpy as np
import torch

from vae2.config import CfgNode

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_TINY = {
    "STAGE1": dict(NUM_MODULES=1, NUM_BRANCHES=1, BLOCK="BOTTLENECK", NUM_BLOCKS=[1],
                   NUM_CHANNELS=[8], FUSE_METHOD="SUM"),
    "STAGE2": dict(NUM_MODULES=1, NUM_BRANCHES=2, BLOCK="BASIC", NUM_BLOCKS=[1, 1],
                   NUM_CHANNELS=[4, 8], FUSE_METHOD="SUM"),
    "STAGE3": dict(NUM_MODULES=1, NUM_BRANCHES=3, BLOCK="BASIC", NUM_BLOCKS=[1, 1, 1],
                   NUM_CHANNELS=[4, 8, 16], FUSE_METHOD="SUM"),
    "STAGE4": dict(NUM_MODULES=1, NUM_BRANCHES=4, BLOCK="BASIC", NUM_BLOCKS=[1, 1, 1, 1],
                   NUM_CHANNELS=[4, 8, 16, 32], FUSE_METHOD="SUM"),
}
_W18 = {
    "STAGE1": dict(NUM_MODULES=1, NUM_BRANCHES=1, BLOCK="BOTTLENECK", NUM_BLOCKS=[2],
                   NUM_CHANNELS=[64], FUSE_METHOD="SUM"),
    "STAGE2": dict(NUM_MODULES=1, NUM_BRANCHES=2, BLOCK="BASIC", NUM_BLOCKS=[2, 2],
                   NUM_CHANNELS=[18, 36], FUSE_METHOD="SUM"),
    "STAGE3": dict(NUM_MODULES=3, NUM_BRANCHES=3, BLOCK="BASIC", NUM_BLOCKS=[2, 2, 2],
                   NUM_CHANNELS=[18, 36, 72], FUSE_METHOD="SUM"),
    "STAGE4": dict(NUM_MODULES=2, NUM_BRANCHES=4, BLOCK="BASIC", NUM_BLOCKS=[2, 2, 2, 2],
                   NUM_CHANNELS=[18, 36, 72, 144], FUSE_METHOD="SUM"),
}


def make_cfg(arch="tiny", hd=False, baseline=False, mode="VAE_NATIVE", z=None, L=3, classes=3,
             hw=(32, 32)):
    st = _TINY if arch == "tiny" else _W18
    extra = dict(IS_BASELINE=baseline, BASELINE_MODE=mode,
                 Z_DIM=z or (4 if arch == "tiny" else 10), HD_Z=hd, FINAL_CONV_KERNEL=1,
                 **copy.deepcopy(st))
    return CfgNode({"MODEL": {"NAME": "enc_hrnet", "PRETRAINED": "", "EXTRA": extra},
                    "DATASET": {"NUM_CLASSES": classes},
                    "TRAIN": {"CLIP_LENGTH": L, "IMAGE_SIZE": [hw[1], hw[0]]}})


def build(cfg, seed=0, with_d=False):
    """ED + EDz (+ the two discriminators with with_d) in tools/train.py's construction
    order (train.py:79-82): returns (ed, ez) or (ed, ez, ds, df)."""
    from vae2 import hrnet
    torch.manual_seed(seed)
    ed = hrnet.get_encdec_model(cfg)
    ez = hrnet.get_encz_model(cfg) if cfg.MODEL.EXTRA.BASELINE_MODE != "DETERMINISTIC" else None
    if not with_d:
        return ed, ez
    return ed, ez, hrnet.get_D_sequence_model(cfg), hrnet.get_D_frame_model(cfg)


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def load_eval_state(g, nets):
    """tiny_eval.npz's trained-looking FullModel_encdec state (sd/<key>) into the modules
    (ez, ed, ds, df) (parameters are copied in place: flat-buffer views stay valid)."""
    prefixes = ("encz_model.", "encdec_model.", "D_model_sequence.", "D_model_frame.")
    for pre, m in zip(prefixes, nets):
        dev = next(m.parameters()).device
        sd = {k[3 + len(pre):]: torch.from_numpy(np.asarray(g[k])).to(dev)
              for k in g.files if k.startswith("sd/" + pre)}
        m.load_state_dict(sd, strict=True)


def ref_checkpoint():
    """The checkpoint the reference itself wrote (make_golden.py ref_ckpt), loaded with a
    loader that executes nothing from the file."""
    return torch.load(os.path.join(GOLDEN, "ref_checkpoint_encdec.pth.tar"), map_location="cpu",
                      weights_only=True)


def t(a):
    return torch.from_numpy(np.asarray(a))


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def rel_nz(a, b):
    """rel(a, b) for a reference that must not be all zero (a lost gradient on both sides
    would otherwise compare equal)."""
    assert b is not None and float(b.detach().double().norm()) > 0, "reference is all zero"
    return rel(a, b)


def max_rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def checksums(sd):
    names = sorted(sd)
    return (np.array([float(sd[k].double().sum()) for k in names]),
            np.array([float(sd[k].double().abs().sum()) for k in names]))
