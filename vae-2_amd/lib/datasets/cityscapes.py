"""Drop-in for the reference's CityscapesSequence (lib/datasets/cityscapes.py:207-326).

Same constructor (root, list_path, ..., crop_size=(H, W), mean, std, clip_length,
clip_num, random_pos, image_tmpl, ...), same list-file and zip format
(tools/gen_cityscapes_data.py:60-88), same window choice and PIL decode/resize.

One deliberate difference: `__getitem__` returns the window as uint8
[clip_length*clip_num][H][W][3] (plus the name) instead of normalised float lists — the
normalisation (cityscapes.py:311-326) runs on the GPU after collation
(`vae2.clips.batch_to_device` / `normalize_clips`, bit-identical to the reference's
numpy), which cuts the host work and the H2D bytes by 4x.  `reference_item` returns the
reference's own ([xt, x2t, x3t], name) structure for callers that need it.

For training at speed, `tools/train.py` uses the decoded uint8 cache + `ClipLoader`
(vae2/clips.py) instead of this per-item PNG decode (MI355X.CLIP_CACHE).
"""
import os

import numpy as np
import torch

from vae2 import clips


class CityscapesSequence(torch.utils.data.Dataset):
    def __init__(self, root, list_path, num_samples=None, num_classes=19, multi_scale=True,
                 flip=True, ignore_label=-1, base_size=2048, crop_size=(512, 1024),
                 center_crop_test=False, downsample_rate=1, scale_factor=16,
                 mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225], clip_length=3,
                 clip_num=3, random_pos=True, image_tmpl="{:06d}_leftImg8bit.png",
                 fixed_length=None, is_baseline=None):
        self.root = root
        self.list_path = list_path
        self.num_classes = num_classes
        self.crop_size = crop_size
        self.mean, self.std = list(mean), list(std)
        self.clip_length = clip_length
        self.clip_num = clip_num
        self.random_pos = random_pos
        self.image_tmpl = image_tmpl
        self.sequence_list = [line.strip() for line in open(list_path)]
        self.files = self.read_files()
        if num_samples:
            self.files = self.files[:num_samples]

    def read_files(self):  # cityscapes.py:269-278
        return [{"seq": p, "name": os.path.splitext(os.path.basename(p))[0]}
                for p in self.sequence_list]

    def __len__(self):
        return len(self.files)

    def get_u8(self, path):
        """uint8 [L*clip_num][H][W][3]: the window cityscapes.py:300-309 reads."""
        n = self.clip_length * self.clip_num
        start = clips.window_start(n, self.random_pos)
        return clips.decode_sequence(os.path.join(self.root, path), self.crop_size,
                                     self.image_tmpl, start, n)

    def __getitem__(self, index):
        item = self.files[index]
        return torch.from_numpy(np.ascontiguousarray(self.get_u8(item["seq"]))), item["name"]

    def reference_item(self, index):
        """([xt, x2t, x3t], name) as float32 CHW arrays, the reference's item structure
        (normalised on the GPU, then copied back)."""
        u8, name = self[index]
        segs = clips.normalize_clips(u8[None].cuda(), self.clip_num, self.mean, self.std)
        return [s[0].cpu().numpy() for s in segs], name
