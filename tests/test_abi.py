"""The C-ABI library loads and exports every entry point include/vae2_hip.h declares
(no compute calls: runs without a GPU)."""
import os
import re

from helpers import GOLDEN  # noqa: F401  (puts the package on sys.path via conftest)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "vae2_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vae2_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from vae2 import _lib
    lib = _lib.load()
    names = declared()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding types every declared entry point, and nothing else
    assert sorted(_lib.exported_symbols()) == names


def test_abi_version_and_error_string():
    from vae2 import _lib
    lib = _lib.load()
    assert lib.vae2_abi_version() == _lib.ABI_VERSION
    assert lib.vae2_last_error() is not None


def test_argument_validation_without_gpu():
    """Bad shapes are rejected on the host (-22) before any launch."""
    import ctypes
    from vae2 import _lib
    lib = _lib.load()
    x = _lib.Act(2, 8, 8, 4, 4)
    y = _lib.Act(2, 5, 8, 4, 4)  # wrong output height for k=3,s=1,p=1
    rc = lib.vae2_conv2d_fwd(ctypes.c_void_p(16), ctypes.byref(x), ctypes.c_void_p(16), None,
                             ctypes.c_void_p(16), ctypes.byref(y), 3, 1, 1, 0.0, None, None)
    assert rc == -22
    assert b"inconsistent conv shapes" in lib.vae2_last_error()
    bad = _lib.Act(2, 8, 8, 4, 2)  # pixel stride < channels
    rc = lib.vae2_bn_stats(ctypes.c_void_p(16), ctypes.byref(bad), ctypes.c_void_p(16), None)
    assert rc == -22
