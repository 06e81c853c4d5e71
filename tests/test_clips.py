"""Clip data path on the CPU: the oracle against the reference's own CityscapesSequence
output (tests/golden/clips.npz), and the host side of vae2.clips (normalisation table,
PNG decode / resize, uint8 cache, window choice, the drop-in dataset) against the
oracle.  The HIP normalisation itself is tested in test_clips_gpu.py."""
import os

import numpy as np
import pytest

from clip_fixtures import case_names, golden, lib_dataset_class, write_case_zip, write_dataset
from oracle import clips_ref


def test_oracle_matches_reference_fixture(tmp_path):
    g = golden()
    crop = tuple(int(v) for v in g["crop_hw"])
    for name in case_names(g):
        zp = write_case_zip(g, name, tmp_path)
        segs = clips_ref.get_item(zp, crop, int(g[f"{name}/start"]), int(g[f"{name}/L"]))
        for i, s in enumerate(segs):
            ref = g[f"{name}/seg{i}"]
            assert s.dtype == np.float32 and s.shape == ref.shape
            assert np.array_equal(s, ref), (name, i)


def test_normalize_table_and_decode_reproduce_reference(tmp_path):
    """uint8 window (vae2.clips.decode_sequence) -> table lookup (normalize_lut) equals
    the reference's float pipeline bit for bit: what the HIP kernel computes."""
    from vae2 import clips
    g = golden()
    crop = tuple(int(v) for v in g["crop_hw"])
    lut = clips.normalize_lut()
    for name in case_names(g):
        zp = write_case_zip(g, name, tmp_path)
        L = int(g[f"{name}/L"])
        start = int(g[f"{name}/start"])
        u8 = clips.decode_sequence(zp, crop, first=start, count=3 * L)
        vals = lut[np.arange(3)[None, None, None, :], u8]  # [F][H][W][3]
        chw = vals.transpose(0, 3, 1, 2).reshape(3 * L * 3, *crop)
        for i in range(3):
            assert np.array_equal(chw[i * 3 * L:(i + 1) * 3 * L], g[f"{name}/seg{i}"]), name


def test_lut_every_byte_against_reference_arithmetic():
    from vae2 import clips
    lut = clips.normalize_lut()
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    # the reference's shapes: an (H, W, 3*n) float32 array, lists tiled n times
    img = np.tile(np.arange(256, dtype=np.float32)[:, None, None], (1, 1, 9))
    x = img / 255.0
    x -= mean * 3
    x /= std * 3
    for c in range(3):
        assert np.array_equal(lut[c], x[:, 0, c])


def test_window_start_rule():
    from vae2 import clips
    assert clips.window_start(9, random_pos=False) == 20
    assert clips.window_start(6, random_pos=False) == 23
    assert clips.window_start(30, random_pos=False) == 0
    np.random.seed(3)
    a = [clips.window_start(9) for _ in range(50)]
    np.random.seed(3)
    b = [clips_ref.window_start(9, True) for _ in range(50)]
    assert a == b and min(a) >= 0 and max(a) <= 21


def test_cache_and_dataset_windows(tmp_path):
    from vae2 import clips
    CityscapesSequence = lib_dataset_class()
    lp = write_dataset(str(tmp_path), 3)
    crop = (16, 32)
    cdir = clips.build_cache(str(tmp_path), lp, crop, workers=1, log=None)
    cache = clips.ClipCache(cdir)
    assert cache.shape == (3, 30, 16, 32, 3)
    assert cache.names == ["seq000", "seq001", "seq002"]
    for i in range(3):
        full = clips.decode_sequence(os.path.join(tmp_path, f"seq{i:03d}.zip"), crop)
        assert np.array_equal(np.asarray(cache.frames[i]), full)
    # reused when unchanged (no rewrite: same mtime)
    m = os.path.getmtime(os.path.join(cdir, "frames.u8"))
    assert clips.build_cache(str(tmp_path), lp, crop, workers=1, log=None) == cdir
    assert os.path.getmtime(os.path.join(cdir, "frames.u8")) == m
    ds = CityscapesSequence(root=str(tmp_path), list_path=lp, num_classes=3, crop_size=crop,
                            random_pos=False)
    assert len(ds) == 3
    u8, name = ds[1]
    assert name == "seq001" and tuple(u8.shape) == (9, 16, 32, 3)
    assert np.array_equal(u8.numpy(), np.asarray(cache.window(1, 20, 9)))


def test_cache_parallel_decode(tmp_path):
    from vae2 import clips
    lp = write_dataset(str(tmp_path), 4, seed=5)
    crop = (8, 16)
    c1 = clips.build_cache(str(tmp_path), lp, crop, cache_dir=str(tmp_path / "c1"), workers=1,
                           log=None)
    c2 = clips.build_cache(str(tmp_path), lp, crop, cache_dir=str(tmp_path / "c2"), workers=2,
                           log=None)
    assert np.array_equal(np.asarray(clips.ClipCache(c1).frames),
                          np.asarray(clips.ClipCache(c2).frames))


def test_incomplete_cache_is_rejected(tmp_path):
    import json
    from vae2 import clips
    lp = write_dataset(str(tmp_path), 1)
    cdir = clips.build_cache(str(tmp_path), lp, (8, 16), workers=1, log=None)
    idx = os.path.join(cdir, "index.json")
    d = json.load(open(idx))
    d["complete"] = False
    json.dump(d, open(idx, "w"))
    with pytest.raises(RuntimeError, match="incomplete"):
        clips.ClipCache(cdir)


def test_metrics_oracle_matches_reference_psnr():
    """oracle/metrics_ref.py's to_image + PSNR / recon against the reference's own PSNR
    (tests/golden/metrics.npz)."""
    from clip_fixtures import GOLDEN_DIR
    from oracle import metrics_ref
    g = np.load(os.path.join(GOLDEN_DIR, "metrics.npz"))
    for k in range(3):
        ia, ib = metrics_ref.to_image(g[f"{k}/a"]), metrics_ref.to_image(g[f"{k}/b"])
        assert abs(metrics_ref.psnr(ia, ib) - float(g[f"{k}/psnr"])) <= 1e-5 * abs(float(g[f"{k}/psnr"]))
        assert abs(metrics_ref.recon_loss(ia, ib) - float(g[f"{k}/recon"])) <= 1e-5 * float(g[f"{k}/recon"])
