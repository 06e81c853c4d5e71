"""Put lib/ (the drop-in package tree) on sys.path, as the reference's tools/_init_paths.py:21-22."""
import os.path as osp
import sys

this_dir = osp.dirname(__file__)
for p in (osp.join(this_dir, "..", "lib"), osp.join(this_dir, "..")):
    if p not in sys.path:
        sys.path.insert(0, p)
