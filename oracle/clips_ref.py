"""ORACLE — test infrastructure only, never on the product path.

numpy / PIL restatement of the reference's clip data path, used by tests/ as the checker
of vae2.clips (uint8 cache + HIP normalisation) and lib/datasets/cityscapes.py:

  CityscapesSequence._load_image   cityscapes.py:290-298  PIL open -> RGB; a frame that
                                                          fails to open falls back to
                                                          idx-1 (idx+1 for frame 0)
  CityscapesSequence.get           cityscapes.py:300-309  window start, resize((W, H)),
                                                          float32
  CityscapesSequence.input_transform  cityscapes.py:311-316  concat on channels, /255,
                                                          -mean, /std (tiled per frame)
  CityscapesSequence.__getitem__   cityscapes.py:318-326  HWC -> CHW, clip_num segments
  zip layout                       gen_cityscapes_data.py:69-83  '{:06d}_<suffix>' members

Pinned by tests/golden/clips.npz, generated from the reference's own CityscapesSequence
(tests/golden/make_golden_clips.py); see tests/test_clips.py.
"""
import zipfile

import numpy as np

FRAMES = 30


def window_start(clip_frames, random_pos, rng=np.random):
    """cityscapes.py:303-304."""
    if random_pos:
        return rng.randint(0, max(1, FRAMES - clip_frames + 1))
    return max(0, FRAMES - clip_frames - 1)


def load_image(zf, idx, tmpl):
    """cityscapes.py:290-298."""
    from PIL import Image
    try:
        return Image.open(zf.open(tmpl.format(idx))).convert("RGB")
    except Exception:
        new_idx = idx - 1 if idx > 0 else idx + 1
        return Image.open(zf.open(tmpl.format(new_idx))).convert("RGB")


def get_item(zip_path, crop_hw, start, clip_length=3, clip_num=3,
             mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
             tmpl="{:06d}_leftImg8bit.png"):
    """The reference's ([xt, x2t, x3t]) for the window starting at `start`:
    list of clip_num float32 [3*clip_length][H][W] arrays."""
    H, W = crop_hw
    n = clip_length * clip_num
    images = []
    with zipfile.ZipFile(zip_path, mode="r") as zf:
        for p in range(start, start + n):
            im = load_image(zf, p, tmpl).resize((W, H))
            images.append(np.asarray(im, dtype=np.float32))
    seq = np.concatenate(images, axis=-1)
    seq = seq / 255.0
    seq -= list(mean) * n
    seq /= list(std) * n
    seq = np.transpose(seq, (2, 0, 1))
    L3 = 3 * clip_length
    return [seq[i * L3:(i + 1) * L3].copy() for i in range(clip_num)]


def write_sequence_zip(path, frames, suffix="leftImg8bit.png", skip=(), modes=None):
    """A sequence zip in the gen_cityscapes_data.py:69-83 layout from uint8 [n][H][W][3]
    frames (PNG members '{:06d}_' + suffix); `skip` leaves members out (missing frames),
    `modes` maps a frame index to the PIL mode it is stored in (e.g. 'RGBA', 'L')."""
    import io
    from PIL import Image
    modes = modes or {}
    with zipfile.ZipFile(path, "w") as zf:
        for i, f in enumerate(frames):
            if i in skip:
                continue
            im = Image.fromarray(f, "RGB")
            if i in modes:
                im = im.convert(modes[i])
            buf = io.BytesIO()
            im.save(buf, format="PNG")
            zf.writestr("{:06d}_{}".format(i, suffix), buf.getvalue())
