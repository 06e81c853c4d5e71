"""Clip input path: Cityscapes sequence zips -> uint8 frame cache -> HBM -> fp32 segments.

Reference data path:
  tools/gen_cityscapes_data.py:60-88  one zip per sequence, 30 frames stored as
                                      '{:06d}_leftImg8bit.png' at 512x256
  cityscapes.py:290-309               window of clip_length*clip_num frames (random start
                                      np.random.randint(0, 30 - L*clip_num + 1), or the
                                      fixed start 30 - L*clip_num - 1), PIL decode ->
                                      RGB -> resize to crop_size -> float32
  cityscapes.py:311-326               concatenate on channels, /255, -mean, /std, HWC ->
                                      CHW, split into clip_num segments of 3*L channels

MI355X design.  PNG decoding cannot feed ~10^3 frames/s per GPU from a few host cores,
and the decode + resize result is the same every time a frame is read (only the window
start is random), so frames are decoded ONCE into a uint8 cache (`build_cache`: one
memory-mapped file [sequences][30][H][W][3] at the crop size, decoded and resized with
PIL exactly as cityscapes.py:292,306 does).  Training reads a window per clip (one
contiguous 9-frame slab copy from the page cache into pinned memory, on a background
thread), uploads the bytes (1/4 of the fp32 tensor) and expands them on the GPU
(`vae2_clip_normalize_u8`: byte -> fp32 table lookup straight into the three segment
tensors).  The normalisation table reproduces the reference's numpy arithmetic bit for
bit (`normalize_lut`), so the segments equal the reference DataLoader's tensors exactly.
"""
import ctypes
import json
import os
import queue
import threading
import zipfile

import numpy as np
import torch

from . import _lib
from .ops import ptr, stream_ptr

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
FRAMES_PER_SEQUENCE = 30
IMAGE_TMPL = "{:06d}_leftImg8bit.png"


# ------------------------------------------------------------ normalisation ----
def normalize_lut(mean=MEAN, std=STD):
    """[3][256] fp32: the value cityscapes.py:311-316 computes for byte v in RGB channel c.

    The reference works on a float32 array: `/ 255.0` stays float32; `-= mean * n` and
    `/= std * n` take float64 lists, so numpy evaluates those two steps in float64 and
    stores float32.  The same sequence of operations, per (channel, byte)."""
    v = np.arange(256, dtype=np.float32)[None, :].repeat(3, 0)
    v = v / 255.0
    v -= np.asarray(mean, dtype=np.float64)[:, None]
    v /= np.asarray(std, dtype=np.float64)[:, None]
    assert v.dtype == np.float32
    return np.ascontiguousarray(v)


_LUTS = {}


def _lut_dev(device, mean, std):
    key = (str(device), tuple(mean), tuple(std))
    t = _LUTS.get(key)
    if t is None:
        t = torch.from_numpy(normalize_lut(mean, std)).to(device)
        _LUTS[key] = t
    return t


def normalize_clips(frames, clip_num=3, mean=MEAN, std=STD, outs=None):
    """frames: uint8 CUDA tensor [B][F][H][W][3] (F = clip_length * clip_num) ->
    list of clip_num fp32 CUDA tensors [B][3F/clip_num][H][W] (the reference's
    [xt, x2t, x3t] batch, cityscapes.py:322-326 after collation)."""
    if frames.dtype != torch.uint8 or frames.dim() != 5 or frames.shape[-1] != 3:
        raise ValueError("frames must be a uint8 tensor [B][F][H][W][3]")
    if not frames.is_cuda:
        raise ValueError("frames must be on the GPU (the normalisation is a HIP kernel)")
    frames = frames.contiguous()
    B, F, H, W, _ = frames.shape
    if F % clip_num:
        raise ValueError(f"{F} frames do not split into {clip_num} segments")
    fs = F // clip_num
    if outs is None:
        outs = [torch.empty((B, 3 * fs, H, W), dtype=torch.float32, device=frames.device)
                for _ in range(clip_num)]
    for o in outs:
        if o.shape != (B, 3 * fs, H, W) or not o.is_contiguous() or o.dtype != torch.float32:
            raise ValueError("bad segment output tensor")
    arr = (ctypes.c_void_p * clip_num)(*[ptr(o) for o in outs])
    _lib.call("vae2_clip_normalize_u8", ptr(frames), B, F, H, W,
              ptr(_lut_dev(frames.device, mean, std)), clip_num, arr, stream_ptr())
    return outs


# ------------------------------------------------------------ window choice ----
def window_start(clip_frames, random_pos=True, rng=np.random):
    """cityscapes.py:303-304 (the same draw from numpy's global generator)."""
    if random_pos:
        return int(rng.randint(0, max(1, FRAMES_PER_SEQUENCE - clip_frames + 1)))
    return max(0, FRAMES_PER_SEQUENCE - clip_frames - 1)


# --------------------------------------------------------------- decoding ----
def decode_sequence(zip_path, crop_hw, image_tmpl=IMAGE_TMPL, first=0,
                    count=FRAMES_PER_SEQUENCE):
    """Frames first..first+count-1 of one sequence zip as uint8 [count][H][W][3], decoded
    and resized as
    cityscapes.py:290-306 does (PIL RGB, Image.resize((W, H)) with PIL's default filter;
    a frame that fails to open is replaced by its predecessor, or frame 1 for frame 0)."""
    from PIL import Image
    H, W = crop_hw
    out = np.empty((count, H, W, 3), dtype=np.uint8)
    with zipfile.ZipFile(zip_path, mode="r") as zf:
        for p in range(first, first + count):
            try:
                im = Image.open(zf.open(image_tmpl.format(p))).convert("RGB")
            except Exception:
                q = p - 1 if p > 0 else p + 1
                im = Image.open(zf.open(image_tmpl.format(q))).convert("RGB")
            out[p - first] = np.asarray(im.resize((W, H)), dtype=np.uint8)
    return out


def _decode_job(args):
    i, path, crop_hw, tmpl, cache_file, shape = args
    mm = np.memmap(cache_file, dtype=np.uint8, mode="r+", shape=shape)
    mm[i] = decode_sequence(path, crop_hw, tmpl)
    mm.flush()
    del mm
    return i


def cache_dir_for(root, list_path, crop_hw):
    base = os.path.splitext(os.path.basename(list_path))[0]
    return os.path.join(root, ".vae2_cache", f"{base}_{crop_hw[0]}x{crop_hw[1]}")


def build_cache(root, list_path, crop_hw, cache_dir=None, workers=None,
                image_tmpl=IMAGE_TMPL, log=print):
    """Decode every sequence zip named in list_path (paths relative to root) once into
    <cache_dir>/frames.u8 ([n][30][H][W][3] uint8) + index.json.  Reuses a complete cache
    whose index matches (list, crop size, zip sizes / mtimes)."""
    cache_dir = cache_dir or cache_dir_for(root, list_path, crop_hw)
    seqs = [line.strip() for line in open(list_path) if line.strip()]
    stamps = []
    for s in seqs:
        st = os.stat(os.path.join(root, s))
        stamps.append([st.st_size, int(st.st_mtime)])
    index = {"version": 1, "sequences": seqs, "names": [os.path.splitext(os.path.basename(s))[0]
                                                         for s in seqs],
             "crop_hw": list(crop_hw), "frames": FRAMES_PER_SEQUENCE, "stamps": stamps,
             "image_tmpl": image_tmpl, "complete": False}
    idx_file = os.path.join(cache_dir, "index.json")
    data_file = os.path.join(cache_dir, "frames.u8")
    if os.path.exists(idx_file):
        with open(idx_file) as f:
            old = json.load(f)
        same = {k: v for k, v in old.items() if k != "complete"} == \
               {k: v for k, v in index.items() if k != "complete"}
        if same and old.get("complete") and os.path.exists(data_file):
            return cache_dir
    os.makedirs(cache_dir, exist_ok=True)
    H, W = crop_hw
    shape = (len(seqs), FRAMES_PER_SEQUENCE, H, W, 3)
    mm = np.memmap(data_file, dtype=np.uint8, mode="w+", shape=shape)
    del mm
    with open(idx_file, "w") as f:
        json.dump(index, f)
    jobs = [(i, os.path.join(root, s), tuple(crop_hw), image_tmpl, data_file, shape)
            for i, s in enumerate(seqs)]
    workers = workers or min(16, len(os.sched_getaffinity(0)))
    if workers > 1 and len(jobs) > 1:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(workers) as pool:
            for k, _ in enumerate(pool.imap_unordered(_decode_job, jobs, chunksize=4)):
                if log and (k + 1) % 100 == 0:
                    log(f"decoded {k + 1}/{len(jobs)} sequences")
    else:
        for j in jobs:
            _decode_job(j)
    index["complete"] = True
    with open(idx_file, "w") as f:
        json.dump(index, f)
    return cache_dir


class ClipCache:
    """Read-only view of a decoded cache: frames[i] is uint8 [30][H][W][3]."""

    def __init__(self, cache_dir):
        with open(os.path.join(cache_dir, "index.json")) as f:
            self.index = json.load(f)
        if not self.index.get("complete"):
            raise RuntimeError(f"clip cache {cache_dir} is incomplete; rebuild it")
        H, W = self.index["crop_hw"]
        self.names = self.index["names"]
        self.shape = (len(self.names), self.index["frames"], H, W, 3)
        self.frames = np.memmap(os.path.join(cache_dir, "frames.u8"), dtype=np.uint8,
                                mode="r", shape=self.shape)

    def __len__(self):
        return self.shape[0]

    def window(self, i, start, count):
        return self.frames[i, start:start + count]


class ClipLoader:
    """Batches of ([xt, x2t, x3t], names) on the GPU from a ClipCache.

    Per batch: indices from `sampler` (a DistributedSampler / RandomSampler, or the
    natural order), one window start per clip (`window_start`, the reference's draw),
    a background thread copies the windows into one of two pinned staging buffers
    (plain slab copies: the GIL is released), the main thread uploads it on a copy
    stream and the HIP kernel expands it on the current stream.  drop_last semantics
    as the reference's DataLoader (train.py:133-140)."""

    def __init__(self, cache, batch_size, clip_length=3, clip_num=3, sampler=None,
                 shuffle=False, random_pos=True, device=None, drop_last=True,
                 mean=MEAN, std=STD, prefetch=2):
        self.cache = cache
        self.B = batch_size
        self.L = clip_length
        self.clip_num = clip_num
        self.F = clip_length * clip_num
        if self.F > cache.shape[1]:
            raise ValueError("clip longer than a cached sequence")
        self.sampler = sampler
        self.shuffle = shuffle
        self.random_pos = random_pos
        self.device = torch.device(device or "cuda")
        self.drop_last = drop_last
        self.mean, self.std = mean, std
        self.prefetch = max(1, prefetch)
        _, _, H, W, _ = cache.shape
        self.staging = [torch.empty((batch_size, self.F, H, W, 3), dtype=torch.uint8,
                                    pin_memory=True) for _ in range(self.prefetch + 1)]
        self._copy_stream = None

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.cache)
        return n // self.B if self.drop_last else -(-n // self.B)

    def _indices(self):
        if self.sampler is not None:
            return list(iter(self.sampler))
        if self.shuffle:
            return torch.randperm(len(self.cache)).tolist()
        return list(range(len(self.cache)))

    def _batches(self):
        idx = self._indices()
        nb = len(self)
        for b in range(nb):
            sel = idx[b * self.B:(b + 1) * self.B]
            starts = [window_start(self.F, self.random_pos) for _ in sel]
            yield sel, starts

    def _fill(self, slot, sel, starts):
        buf = self.staging[slot].numpy()
        for k, (i, s) in enumerate(zip(sel, starts)):
            buf[k] = self.cache.window(i, s, self.F)
        return len(sel)

    def __iter__(self):
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=self.device)
        q = queue.Queue(maxsize=self.prefetch)
        plan = list(self._batches())
        stop = threading.Event()
        free = queue.Queue()
        for s in range(len(self.staging)):
            free.put(s)

        def producer():
            try:
                for sel, starts in plan:
                    slot = free.get()
                    if stop.is_set():
                        return
                    n = self._fill(slot, sel, starts)
                    q.put((slot, n, sel))
            except BaseException as e:  # surface worker errors in the consumer
                q.put(e)
                return
            q.put(None)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        pending = None  # (slot, event) whose staging buffer frees once the H2D is done
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                slot, n, sel = item
                cur = torch.cuda.current_stream(self.device)
                with torch.cuda.stream(self._copy_stream):
                    self._copy_stream.wait_stream(cur)  # the dev buffer may still be read
                    dev = self.staging[slot][:n].to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._copy_stream)
                cur.wait_event(ev)
                dev.record_stream(cur)
                segs = normalize_clips(dev, self.clip_num, self.mean, self.std)
                if pending is not None:
                    pending[1].synchronize()
                    free.put(pending[0])
                pending = (slot, ev)
                names = [self.cache.names[i] for i in sel]
                yield segs, names
        finally:
            stop.set()
            if pending is not None:
                pending[1].synchronize()
                free.put(pending[0])
            for s in range(len(self.staging)):
                free.put(s)
            th.join(timeout=10)


def batch_to_device(xs, device, clip_num=3):
    """A loader batch's clips on the device as [xt, x2t, x3t]: a uint8 window batch
    ([B][F][H][W][3], what lib/datasets/cityscapes.CityscapesSequence yields) goes
    through the HIP normalisation; fp32 segment lists (already normalised, e.g. the
    synthetic clips or a ClipLoader batch) are moved as they are."""
    if torch.is_tensor(xs) and xs.dtype == torch.uint8:
        return normalize_clips(xs.to(device, non_blocking=True), clip_num)
    return [x.to(device) for x in xs]
