"""Generate tests/golden/clips.npz: the reference's own CityscapesSequence output on
synthetic sequence zips.  Runs ONLY in the build container (it imports
/root/reference/lib/datasets/cityscapes.py read-only and writes data only).

Shims (not edits of the reference): `cv2` is imported at the top of cityscapes.py /
base_dataset.py but not used by the sequence path, so an empty module stands in for it;
the object is made with object.__new__ and the attributes __init__ would set, because
__init__ moves a class-weight tensor to CUDA (cityscapes.py:236-240), absent here.

Cases (source frames 24x48 uint8, 30 per zip, crop (16, 32) so PIL's resize runs):
  fixed      random_pos=False: start 30 - 9 - 1 = 20 (cityscapes.py:304)
  random     random_pos=True after np.random.seed(7): the window start is recorded
  fallback   frames 0 and 21 missing from the zip (cityscapes.py:293-296 falls back to
             frame 1 / frame 20), frame 22 stored as RGBA and 23 as L (convert('RGB'))
  l2         clip_length 2, clip_num 3 (BASELINE config 2 frame layout), fixed start
Stored: the source frames (tests rebuild the zips from them: PNG is lossless), the
missing / mode lists, the window start, and the reference's three segment arrays.

    python tests/golden/make_golden_clips.py
"""
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/lib"

CASES = {
    "fixed": dict(random_pos=False, L=3, skip=(), modes={}),
    "random": dict(random_pos=True, L=3, skip=(), modes={}, seed=7),
    "fallback": dict(random_pos=False, L=3, skip=(0, 21), modes={22: "RGBA", 23: "L"}),
    "l2": dict(random_pos=False, L=2, skip=(), modes={}),
}
SRC_HW = (24, 48)
CROP = (16, 32)


def main():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, REF)
    sys.path.insert(0, REPO)
    from datasets.cityscapes import CityscapesSequence  # the reference's class
    from oracle.clips_ref import write_sequence_zip

    out = {}
    rng = np.random.RandomState(1234)
    with tempfile.TemporaryDirectory() as td:
        for name, c in CASES.items():
            frames = rng.randint(0, 256, size=(30,) + SRC_HW + (3,), dtype=np.uint8)
            zname = f"seq_{name}.zip"
            write_sequence_zip(os.path.join(td, zname), frames, skip=c["skip"], modes=c["modes"])
            ds = object.__new__(CityscapesSequence)
            ds.root = td
            ds.crop_size = CROP
            ds.mean = [0.485, 0.456, 0.406]
            ds.std = [0.229, 0.224, 0.225]
            ds.clip_length = c["L"]
            ds.clip_num = 3
            ds.random_pos = c["random_pos"]
            ds.image_tmpl = "{:06d}_leftImg8bit.png"
            ds.files = [{"seq": zname, "name": zname[:-4]}]
            if c["random_pos"]:
                np.random.seed(c["seed"])
                start = np.random.randint(0, max(1, 30 - c["L"] * 3 + 1))
                np.random.seed(c["seed"])
            else:
                start = max(0, 30 - c["L"] * 3 - 1)
            segs, nm = CityscapesSequence.__getitem__(ds, 0)
            assert nm == zname[:-4]
            out[f"{name}/frames"] = frames
            out[f"{name}/skip"] = np.asarray(c["skip"], dtype=np.int64)
            out[f"{name}/modes"] = np.asarray([[k, {"RGBA": 1, "L": 2}[v]]
                                              for k, v in c["modes"].items()],
                                             dtype=np.int64).reshape(-1, 2)
            out[f"{name}/L"] = np.int64(c["L"])
            out[f"{name}/start"] = np.int64(start)
            for i, s in enumerate(segs):
                out[f"{name}/seg{i}"] = np.asarray(s, dtype=np.float32)
    out["crop_hw"] = np.asarray(CROP, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "clips.npz"), **out)
    print("wrote", os.path.join(HERE, "clips.npz"), sorted(out)[:6], "...")


if __name__ == "__main__":
    main()
