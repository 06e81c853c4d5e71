"""Clip input-path throughput: can the data path feed the training step?

Writes `--seqs` synthetic sequence zips in the reference's on-disk format (30 PNG frames
at the stored 512x256, gen_cityscapes_data.py:60-88), then measures
  decode   the reference-style per-item path (PIL decode + resize of a 9-frame window)
  cache    building the uint8 frame cache (all frames decoded once, `--workers`)
  loader   ClipLoader batches (window copy -> pinned -> H2D -> vae2_clip_normalize_u8)
  kernel   vae2_clip_normalize_u8 alone (HIP events): us per batch and GB/s
and prints one JSON line.  Frames/s counts the 3*L frames a clip ingests (bench.py's unit).

    python vae-2_amd/tools/clip_bench.py --seqs 32 --height 128 --width 256 --batch 8
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from vae2 import clips  # noqa: E402


def write_zips(root, n, stored_hw=(256, 512), seed=0):
    import io
    import zipfile
    from PIL import Image
    rng = np.random.RandomState(seed)
    H, W = stored_hw
    # smooth-ish images (PNG size / decode cost closer to real frames than white noise)
    yy, xx = np.mgrid[0:H, 0:W]
    names = []
    for i in range(n):
        nm = f"seq{i:04d}.zip"
        with zipfile.ZipFile(os.path.join(root, nm), "w") as zf:
            for f in range(30):
                ph = rng.uniform(0, 6.28, 3)
                img = np.stack([127 + 100 * np.sin(xx / (17 + 5 * c) + yy / 23 + ph[c] + f / 5)
                                for c in range(3)], -1)
                img = (img + rng.randint(0, 8, img.shape)).clip(0, 255).astype(np.uint8)
                buf = io.BytesIO()
                Image.fromarray(img).save(buf, format="PNG")
                zf.writestr("{:06d}_leftImg8bit.png".format(f), buf.getvalue())
        names.append(nm)
    lp = os.path.join(root, "list.text")
    with open(lp, "w") as f:
        f.write("\n".join(names))
    return lp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=32)
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--clip-length", type=int, default=3)
    ap.add_argument("--workers", type=int, default=min(16, len(os.sched_getaffinity(0))))
    ap.add_argument("--epochs", type=int, default=4)
    args = ap.parse_args()
    crop = (args.height, args.width)
    F = 3 * args.clip_length
    res = {"seqs": args.seqs, "crop_hw": list(crop), "batch": args.batch, "frames_per_clip": F,
           "workers": args.workers}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as root:
        t = time.perf_counter()
        lp = write_zips(root, args.seqs)
        res["write_s"] = round(time.perf_counter() - t, 2)
        # reference-style per-item decode (one process)
        t = time.perf_counter()
        n = min(8, args.seqs)
        for i in range(n):
            clips.decode_sequence(os.path.join(root, f"seq{i:04d}.zip"), crop, first=20, count=F)
        res["decode_item_frames_per_s_1proc"] = round(n * F / (time.perf_counter() - t), 1)
        t = time.perf_counter()
        cdir = clips.build_cache(root, lp, crop, workers=args.workers, log=None)
        dt = time.perf_counter() - t
        res["cache_build_s"] = round(dt, 2)
        res["cache_decode_frames_per_s"] = round(args.seqs * 30 / dt, 1)
        cache = clips.ClipCache(cdir)
        _ = np.asarray(cache.frames).sum()  # page the cache in (steady state: page cache)
        loader = clips.ClipLoader(cache, args.batch, clip_length=args.clip_length, shuffle=True,
                                  device="cuda")
        for segs, _ in loader:  # warm-up
            pass
        torch.cuda.synchronize()
        t = time.perf_counter()
        nb = 0
        for _ in range(args.epochs):
            for segs, _ in loader:
                nb += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        res["loader_batches"] = nb
        res["loader_frames_per_s"] = round(nb * args.batch * F / dt, 1)
        # the kernel alone
        u8 = torch.randint(0, 256, (args.batch, F) + crop + (3,), dtype=torch.uint8,
                           device="cuda")
        outs = [torch.empty((args.batch, 3 * args.clip_length) + crop, device="cuda")
                for _ in range(3)]
        for _ in range(5):
            clips.normalize_clips(u8, 3, outs=outs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 50
        for _ in range(reps):
            clips.normalize_clips(u8, 3, outs=outs)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / reps
        bytes_ = u8.numel() * 5  # 1 B read + 4 B written per element
        res["kernel_us"] = round(us, 2)
        res["kernel_gbs"] = round(bytes_ / us / 1e3, 1)
        res["kernel_frac_hbm_peak"] = round(bytes_ / us / 1e3 / 8000, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
