"""Build libvae2_hip.so (gfx950) from the HIP sources in this directory.

Plain hipcc invocations, one object per source compiled in parallel, then one
shared-library link.  The library lands next to the Python package
(vae-2_amd/vae2/libvae2_hip.so) so it travels with the repo snapshot.
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "vae2")
# A/B builds: VAE2_BUILD_TAG=t VAE2_DEFS="-DVAE2_ABLATE=1" -> libvae2_hip_t.so (own objects)
TAG = os.environ.get("VAE2_BUILD_TAG", "")
DEFS = os.environ.get("VAE2_DEFS", "").split()
OUT = os.path.join(PKG, f"libvae2_hip_{TAG}.so" if TAG else "libvae2_hip.so")
BUILD = os.path.join(HERE, f"build_{TAG}" if TAG else "build")
SOURCES = ["conv.hip", "bn.hip", "resample.hip", "elbo.hip", "heads.hip", "clips.hip",
           "metrics.hip", "wgrad_narrow.hip", "syncbn.hip", "dconv_stream.hip"]
HEADERS = ["common.h", os.path.join("..", "..", "include", "vae2_hip.h")]
ARCH = os.environ.get("VAE2_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
         "-Wno-unused-function", "-munsafe-fp-atomics"]
# per-source extras: no SLP vectorisation in the conv kernels (it packs independent f32
# FMAs beside the MFMAs into v_pk_fma_f32 + operand moves, which cost issue slots there)
EXTRA = {"conv.hip": ["-fno-slp-vectorize"], "dconv_stream.hip": ["-fno-slp-vectorize"]}
# conv.hip is compiled as four objects (VAE2_CONV_PART 0..3: pack + C-ABI dispatch, gather
# kernels, direct 3x3 kernels, weight-gradient kernels) so its instantiations build in
# parallel
PARTS = {"conv.hip": 4}


def _units():
    out = []
    for src in SOURCES:
        n = PARTS.get(src, 0)
        base = os.path.splitext(src)[0]
        if n:
            out += [(src, f"{base}_p{i}.o", [f"-DVAE2_CONV_PART={i}"]) for i in range(n)]
        else:
            out.append((src, base + ".o", []))
    return out


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(unit):
    src, oname, defs = unit
    obj = os.path.join(BUILD, oname)
    deps = [os.path.join(HERE, src)] + [os.path.join(HERE, h) for h in HEADERS]
    if not _newer(obj, deps):
        return obj, None
    cmd = [hipcc()] + FLAGS + EXTRA.get(src, []) + defs + DEFS + ["-c", os.path.join(HERE, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(verbose=True, force=False):
    os.makedirs(BUILD, exist_ok=True)
    if force:
        for f in os.listdir(BUILD):
            os.remove(os.path.join(BUILD, f))
    units = _units()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(units))) as ex:
        results = list(ex.map(_compile, units))
    errors = [e for _, e in results if e]
    if errors:
        raise RuntimeError("HIP compile failed:\n" + "\n".join(errors))
    objs = [o for o, _ in results]
    if force or _newer(OUT, objs):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {OUT}")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
