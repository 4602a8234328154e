"""In-tree build of libqce.so (hipcc, gfx950 only).

``python -m quantized_channel_estimation_amd.build`` compiles every ``csrc/*.hip`` to an object
in ``build/`` and links ``quantized_channel_estimation_amd/libqce.so``.  Objects are rebuilt
only when a source or header is newer.  The .so is git-ignored but travels to the GPU box
with the repository snapshot.
"""
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "qce")
LIB = os.path.join(PKG, "libqce.so")
ARCH = "gfx950"


def _hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP library cannot be built")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, jobs=None, variant=None):
    """variant "stamps": diagnostic library libqce_stamps.so compiled with -DQCE_STAMPS."""
    hipcc = _hipcc()
    build_dir = BUILD if variant is None else BUILD + "_" + variant
    lib_path = LIB if variant is None else os.path.join(PKG, f"libqce_{variant}.so")
    os.makedirs(build_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "qce.h")]
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
             "-I" + os.path.join(ROOT, "include")]
    if variant == "stamps":
        flags.append("-DQCE_STAMPS")

    def compile_one(src):
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        if _newer(obj, [src] + headers):
            cmd = [hipcc] + flags + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-4000:]}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    if _newer(lib_path, objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    return lib_path


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, variant="stamps" if "--stamps" in sys.argv else None))
