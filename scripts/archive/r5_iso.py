"""Isolate the conv_bn_train[True-False-1-18] failure: run it under tune keys 7 / 8."""
import sys
sys.path[:0] = ["tests", "vae-2_amd", "."]
import torch  # noqa
from vae2 import _lib
import test_kernels_gpu as T
lib = _lib.load()
for k7, k8 in ((1, 1), (0, 1), (1, 0), (0, 0)):
    lib.vae2_conv2d_set_tune(7, k7)
    lib.vae2_conv2d_set_tune(8, k8)
    try:
        T.test_conv_bn_train(True, False, 1, 18)
        print(k7, k8, "pass", flush=True)
    except AssertionError as e:
        print(k7, k8, "FAIL", str(e)[:200].replace("\n", " "), flush=True)
