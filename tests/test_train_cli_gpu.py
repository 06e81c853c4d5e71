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


def _train(tmp_path, *opts):
    if TOOLS not in sys.path:
        sys.path.insert(0, TOOLS)
    import train  # vae-2_amd/tools/train.py
    from config import config
    config.defrost()
    config.merge_from_file(YAML)  # reset anything a previous run merged
    config.freeze()
    argv = ["--cfg", YAML, "OUTPUT_DIR", str(tmp_path / "output"), "LOG_DIR", str(tmp_path / "log"),
            "TRAIN.IMAGE_SIZE", "[64, 32]", "TRAIN.BATCH_SIZE_PER_GPU", "2",
            "MI355X.SYNTHETIC_CLIPS", "4", "PRINT_FREQ", "1", "MI355X.DEFER_CHECKS", "True",
            *opts]
    train.main(argv)
    return os.path.join(str(tmp_path / "output"), "cityscapessequence",
                        os.path.basename(YAML).split(".")[0])


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
