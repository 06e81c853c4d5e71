"""Clip data path on the GPU: vae2_clip_normalize_u8 (through vae2.clips) against the
reference's own CityscapesSequence output (tests/golden/clips.npz) and the oracle,
bit for bit; the cached ClipLoader batches; the uint8 DataLoader path."""
import numpy as np
import pytest
import torch

from clip_fixtures import case_names, golden, lib_dataset_class, write_case_zip, write_dataset
from oracle import clips_ref

pytestmark = pytest.mark.gpu


def test_normalize_kernel_equals_reference_fixture(tmp_path):
    from vae2 import clips
    g = golden()
    crop = tuple(int(v) for v in g["crop_hw"])
    by_L = {}
    for name in case_names(g):
        zp = write_case_zip(g, name, tmp_path)
        L = int(g[f"{name}/L"])
        u8 = clips.decode_sequence(zp, crop, first=int(g[f"{name}/start"]), count=3 * L)
        by_L.setdefault(L, []).append((name, u8))
    for L, items in by_L.items():
        batch = torch.from_numpy(np.stack([u for _, u in items])).cuda()
        segs = clips.normalize_clips(batch, 3)
        torch.cuda.synchronize()
        for b, (name, _) in enumerate(items):
            for i in range(3):
                got = segs[i][b].cpu().numpy()
                assert np.array_equal(got, g[f"{name}/seg{i}"]), (name, i)


@pytest.mark.parametrize("crop,L,clip_num", [((15, 31), 3, 3), ((16, 30), 2, 3),
                                             ((32, 64), 4, 2), ((7, 9), 1, 1)])
def test_normalize_kernel_shapes(tmp_path, crop, L, clip_num):
    """Quad path (h*w % 4 == 0) and per-pixel path, other segment counts."""
    from vae2 import clips
    rng = np.random.RandomState(sum(crop) + L)
    B, F = 3, L * clip_num
    u8 = rng.randint(0, 256, size=(B, F) + crop + (3,), dtype=np.uint8)
    segs = clips.normalize_clips(torch.from_numpy(u8).cuda(), clip_num)
    lut = clips.normalize_lut()
    ref = lut[np.arange(3)[None, None, None, None, :], u8]  # [B][F][H][W][3]
    ref = ref.transpose(0, 1, 4, 2, 3).reshape(B, 3 * F, *crop)
    fs3 = 3 * L
    for i in range(clip_num):
        assert np.array_equal(segs[i].cpu().numpy(), ref[:, i * fs3:(i + 1) * fs3])


def test_normalize_rejects_bad_input():
    from vae2 import clips
    with pytest.raises(ValueError):
        clips.normalize_clips(torch.zeros((1, 9, 4, 4, 3), dtype=torch.uint8), 3)  # host
    with pytest.raises(ValueError):
        clips.normalize_clips(torch.zeros((1, 8, 4, 4, 3), dtype=torch.uint8).cuda(), 3)
    with pytest.raises(ValueError):
        clips.normalize_clips(torch.zeros((1, 9, 4, 4, 3)).cuda(), 3)


@pytest.mark.parametrize("random_pos", [False, True])
def test_clip_loader_batches_equal_oracle(tmp_path, random_pos):
    from vae2 import clips
    lp = write_dataset(str(tmp_path), 5, seed=11)
    crop = (16, 32)
    cache = clips.ClipCache(clips.build_cache(str(tmp_path), lp, crop, workers=1, log=None))
    loader = clips.ClipLoader(cache, batch_size=2, random_pos=random_pos, device="cuda")
    assert len(loader) == 2  # drop_last
    np.random.seed(5)
    got = [([s.cpu().numpy() for s in segs], names) for segs, names in loader]
    np.random.seed(5)
    starts = [clips_ref.window_start(9, random_pos) for _ in range(4)]
    k = 0
    for segs, names in got:
        assert len(segs) == 3 and segs[0].shape == (2, 9) + crop
        for b, nm in enumerate(names):
            zp = str(tmp_path / f"{nm}.zip")
            ref = clips_ref.get_item(zp, crop, starts[k])
            k += 1
            for i in range(3):
                assert np.array_equal(segs[i][b], ref[i]), (nm, i)
    assert [n for _, ns in got for n in ns] == ["seq000", "seq001", "seq002", "seq003"]


def test_clip_loader_with_distributed_sampler_and_epochs(tmp_path):
    from vae2 import clips
    lp = write_dataset(str(tmp_path), 6, seed=2)
    cache = clips.ClipCache(clips.build_cache(str(tmp_path), lp, (8, 16), workers=1, log=None))
    seen = []
    for rank in range(2):
        s = torch.utils.data.distributed.DistributedSampler(list(range(6)), num_replicas=2,
                                                            rank=rank, shuffle=True, seed=0)
        s.set_epoch(1)
        ld = clips.ClipLoader(cache, batch_size=1, sampler=s, random_pos=False, device="cuda")
        names = [n for _ in range(2) for _, ns in ld for n in ns]  # two passes: re-iterable
        assert len(names) == 6
        seen += names[:3]
        assert names[:3] == names[3:]
    assert sorted(seen) == [f"seq{i:03d}" for i in range(6)]


def test_u8_dataloader_path_equals_reference_items(tmp_path):
    """lib/datasets CityscapesSequence through a torch DataLoader (uint8 windows) ->
    batch_to_device == the reference's items stacked."""
    from vae2 import clips
    lp = write_dataset(str(tmp_path), 4, seed=3)
    crop = (16, 32)
    ds = lib_dataset_class()(root=str(tmp_path), list_path=lp, crop_size=crop, random_pos=False)
    dl = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False, num_workers=0,
                                     drop_last=True)
    for bi, (xs, names) in enumerate(dl):
        segs = clips.batch_to_device(xs, "cuda")
        for b, nm in enumerate(names):
            ref = clips_ref.get_item(str(tmp_path / f"{nm}.zip"), crop, 20)
            for i in range(3):
                assert np.array_equal(segs[i][b].cpu().numpy(), ref[i])
