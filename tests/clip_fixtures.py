"""Shared fixtures of the clip-path tests: rebuild the golden sequence zips."""
import os

import numpy as np

from helpers import GOLDEN
from oracle.clips_ref import write_sequence_zip

MODES = {1: "RGBA", 2: "L"}
GOLDEN_DIR = GOLDEN


def lib_dataset_class():
    """vae-2_amd/lib/datasets/cityscapes.py's CityscapesSequence (loaded by path: the
    top-level name `datasets` is also an installed Hugging Face package)."""
    import importlib.util
    path = os.path.join(os.path.dirname(GOLDEN), "..", "vae-2_amd", "lib", "datasets",
                        "cityscapes.py")
    spec = importlib.util.spec_from_file_location("vae2_lib_datasets_cityscapes", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CityscapesSequence


def golden():
    return np.load(os.path.join(GOLDEN, "clips.npz"))


def case_names(g):
    return sorted({k.split("/")[0] for k in g.files if "/" in k})


def write_case_zip(g, name, directory):
    path = os.path.join(directory, f"seq_{name}.zip")
    modes = {int(k): MODES[int(v)] for k, v in g[f"{name}/modes"]}
    write_sequence_zip(path, g[f"{name}/frames"], skip=set(g[f"{name}/skip"].tolist()),
                       modes=modes)
    return path


def write_dataset(directory, n, hw=(24, 48), seed=0, list_name="train_list.text"):
    """n random sequence zips + a list file (paths relative to the root, as
    gen_cityscapes_data.py writes them)."""
    rng = np.random.RandomState(seed)
    names = []
    for i in range(n):
        frames = rng.randint(0, 256, size=(30,) + tuple(hw) + (3,), dtype=np.uint8)
        nm = f"seq{i:03d}.zip"
        write_sequence_zip(os.path.join(directory, nm), frames)
        names.append(nm)
    lp = os.path.join(directory, list_name)
    with open(lp, "w") as f:
        f.write("\n".join(names))
    return lp
