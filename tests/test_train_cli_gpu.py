"""The drop-in CLI (vae-2_amd/tools/train.py) end to end on the GPU: YAML + KEY VALUE
overrides -> models -> FullModel_encdec / FullModel_D -> adversarial_train epochs ->
the reference's checkpoint files and state_dict keys (train.py:317-348) -> TRAIN.RESUME
(train.py:270-290)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "vae-2_amd", "tools")
YAML = os.path.join(ROOT, "vae-2_amd", "experiments", "vae2_w18_small_v2_128x256.yaml")

pytestmark = pytest.mark.gpu


def _train(tmp_path, *opts, cfg=YAML, size="[64, 32]"):
    if TOOLS not in sys.path:
        sys.path.insert(0, TOOLS)
    import train  # vae-2_amd/tools/train.py
    from config import config
    config.defrost()
    config.merge_from_file(cfg)  # reset anything a previous run merged
    config.freeze()
    argv = ["--cfg", cfg, "OUTPUT_DIR", str(tmp_path / "output"), "LOG_DIR", str(tmp_path / "log"),
            "TRAIN.IMAGE_SIZE", size, "TRAIN.BATCH_SIZE_PER_GPU", "2",
            "MI355X.SYNTHETIC_CLIPS", "4", "PRINT_FREQ", "1", "MI355X.DEFER_CHECKS", "True",
            *opts]
    train.main(argv)
    return os.path.join(str(tmp_path / "output"), "cityscapessequence",
                        os.path.basename(cfg).split(".")[0])


def test_train_cli_elbo_checkpoint_and_resume(tmp_path):
    out = _train(tmp_path, "TRAIN.END_EPOCH", "1", "MI355X.ELBO_ONLY", "True")
    ck = torch.load(os.path.join(out, "checkpoint_encdec.pth.tar"), map_location="cpu",
                    weights_only=True)
    assert ck["epoch"] == 1
    keys = list(ck["state_dict"])
    assert any(k.startswith("encz_model.") for k in keys)
    assert any(k.startswith("encdec_model.decf_") for k in keys)
    assert "encdec_model.bn1.running_var" in keys
    assert all(torch.isfinite(v).all() for v in ck["state_dict"].values() if v.is_floating_point())
    assert os.path.isfile(os.path.join(out, "model_encdec_final_state.pth"))
    assert len(ck["optimizer_encdec"]["state"]) == len([k for k in keys if not any(
        s in k for s in ("running_", "num_batches"))])
    # resume: one more epoch starting from the saved one
    _train(tmp_path, "TRAIN.END_EPOCH", "2", "MI355X.ELBO_ONLY", "True", "TRAIN.RESUME", "True")
    ck2 = torch.load(os.path.join(out, "checkpoint_encdec.pth.tar"), map_location="cpu",
                     weights_only=True)
    assert ck2["epoch"] == 2
    st = ck2["optimizer_encdec"]["state"]
    assert int(float(st[0]["step"])) == 4  # 2 iterations per epoch x 2 epochs
    w1 = ck["state_dict"]["encdec_model.conv1.weight"]
    w2 = ck2["state_dict"]["encdec_model.conv1.weight"]
    assert not torch.equal(w1, w2)


def test_train_cli_full_vae2_gan_step(tmp_path):
    """GAN_LAMBDA 1 with both discriminators and the D step (the reference default)."""
    out = _train(tmp_path, "TRAIN.END_EPOCH", "1", "TRAIN.GAN_LAMBDA", "1.0", "MI355X.ELBO_ONLY", "False")
    ck = torch.load(os.path.join(out, "checkpoint_encdec.pth.tar"), map_location="cpu",
                    weights_only=True)
    keys = list(ck["state_dict"])
    assert any(k.startswith("D_model_sequence.") for k in keys)
    assert any(k.startswith("D_model_frame.last_layer.") for k in keys)
    ckd = torch.load(os.path.join(out, "checkpoint_D.pth.tar"), map_location="cpu",
                     weights_only=True)
    assert ckd["epoch"] == 1 and "optimizer_D" in ckd
    assert any(k.startswith("D_model_sequence.") for k in ckd["state_dict"])
    assert os.path.isfile(os.path.join(out, "model_D_final_state.pth"))
    d_state = ckd["optimizer_D"]["state"]
    assert int(float(d_state[0]["step"])) == 2


@pytest.mark.parametrize("cache", [True, False])
def test_train_and_inference_cli_on_sequence_zips(tmp_path, cache):
    """The Cityscapes sequence-zip data path end to end: tools/train.py on 4 zips
    (uint8 cache + ClipLoader, or the drop-in CityscapesSequence through a DataLoader),
    then tools/inference.py (prior sampling, eval metrics) from the saved checkpoint."""
    import numpy as np
    from PIL import Image
    from clip_fixtures import write_dataset
    from vae2 import clips
    data = tmp_path / "data"
    data.mkdir()
    lp = write_dataset(str(data), 4, hw=(24, 48), seed=4)
    opts = ["DATASET.ROOT", str(data), "DATASET.TRAIN_SET", lp, "MI355X.SYNTHETIC_DATA", "False",
            "MI355X.CLIP_CACHE", str(cache), "MI355X.ELBO_ONLY", "True"]
    out = _train(tmp_path, "TRAIN.END_EPOCH", "1", *opts)
    ck = torch.load(os.path.join(out, "checkpoint_encdec.pth.tar"), map_location="cpu",
                    weights_only=True)
    assert ck["epoch"] == 1
    assert int(float(ck["optimizer_encdec"]["state"][0]["step"])) == 2  # 4 clips / B=2
    assert os.path.isdir(os.path.join(str(data), ".vae2_cache")) == cache

    import inference  # vae-2_amd/tools/inference.py (tools/ is on sys.path after _train)
    from config import config
    config.defrost()
    config.merge_from_file(YAML)
    config.freeze()
    res = inference.main(["--cfg", YAML, "OUTPUT_DIR", str(tmp_path / "output"),
                          "LOG_DIR", str(tmp_path / "log"), "TRAIN.IMAGE_SIZE", "[64, 32]",
                          "TRAIN.BATCH_SIZE_PER_GPU", "2", "TRAIN.RESUME", "True",
                          "MI355X.EVAL_SAMPLES", "2", *opts])
    assert [r[0] for r in res] == ["seq001", "seq003"]  # the last clip of each batch
    vis = os.path.join(out, "vis", "epoch0", "seq001")
    # ground-truth frames: to_image(normalise(u8)) truncated to uint8 is the window again
    u8 = clips.decode_sequence(os.path.join(str(data), "seq001.zip"), (32, 64), first=20,
                               count=9)
    for k, tag in enumerate(("x1t", "x2t", "x3t")):
        for i in range(3):
            png = np.asarray(Image.open(os.path.join(vis, f"{tag}_{i}.png")))
            assert np.abs(png.astype(int) - u8[3 * k + i].astype(int)).max() <= 1
    per = dict(res[0][1])
    for tag in ("x2t", "x3t"):
        m = per[tag]
        assert m.shape == (2, 3, 4)
        assert np.isfinite(m[..., [0, 1, 3]]).all() and np.isnan(m[..., 2]).all()
        assert ((m[..., 1] > -1) & (m[..., 1] <= 1)).all()
        lines = open(os.path.join(vis, f"{tag}predict", f"{tag}_0_ssimloss.txt")).read().split()
        assert len(lines) == 2 and abs(float(lines[1]) - m[1, 0, 1]) < 1e-6
        pngs = [f for f in os.listdir(os.path.join(vis, f"{tag}predict")) if f.endswith(".png")]
        assert len(pngs) == 2 * 3


def test_train_cli_resumes_a_reference_checkpoint(tmp_path):
    """TRAIN.RESUME (train.py:270-290) from checkpoint_encdec.pth.tar as the reference
    itself writes it (tests/golden/ref_checkpoint_encdec.pth.tar: the tiny HRNet after one
    Adam step, discriminator keys included): the run continues at epoch 1 with the saved
    Adam moments (step counter 1 + 2 iterations)."""
    import shutil
    import yaml
    from helpers import _TINY, GOLDEN
    with open(YAML) as f:
        cfg = yaml.safe_load(f)
    cfg["MODEL"]["EXTRA"].update({k: dict(v) for k, v in _TINY.items()})
    cfg["MODEL"]["EXTRA"]["Z_DIM"] = 4
    tiny = str(tmp_path / "vae2_tiny.yaml")
    with open(tiny, "w") as f:
        yaml.safe_dump(cfg, f)
    out = tmp_path / "output" / "cityscapessequence" / "vae2_tiny"
    out.mkdir(parents=True)
    shutil.copy(os.path.join(GOLDEN, "ref_checkpoint_encdec.pth.tar"),
                str(out / "checkpoint_encdec.pth.tar"))
    ref = torch.load(str(out / "checkpoint_encdec.pth.tar"), map_location="cpu", weights_only=True)
    _train(tmp_path, "TRAIN.END_EPOCH", "2", "TRAIN.RESUME", "True", "MI355X.ELBO_ONLY", "True",
           cfg=tiny, size="[32, 32]")
    ck = torch.load(str(out / "checkpoint_encdec.pth.tar"), map_location="cpu", weights_only=True)
    assert ck["epoch"] == 2
    assert int(float(ck["optimizer_encdec"]["state"][0]["step"])) == 3
    assert set(ck["state_dict"]) == {k for k in ref["state_dict"] if not k.startswith("D_model")}
    w0 = ref["state_dict"]["encdec_model.conv1.weight"]
    w1 = ck["state_dict"]["encdec_model.conv1.weight"]
    assert not torch.equal(w0, w1) and float((w1 - w0).abs().max()) < 1e-3  # 2 Adam steps
