"""Build recipe for the gfx950 C-ABI library ``gsvc_amd/lib/libgsvc_amd.so``.

    python -m gsvc_amd.build            # or __graft_entry__.build()

One ``hipcc --offload-arch=gfx950`` compile per ``.hip`` source (object files
cached under gsvc_amd/lib/obj by mtime), then one shared-object link.  The
library is built in-tree so it travels to the GPU box with the repo snapshot.
``-ffp-contract=off`` fixes the floating-point op sequence (every fused
multiply-add in the kernels is an explicit ``fmaf``), which the CPU oracle
restates; see DESIGN.md §4.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libgsvc_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC", "-std=c++17",
         "-Wall", "-Wno-unused-result"]


def _deps():
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + [
        os.path.join(os.path.dirname(HERE), "include", "gsvc_amd.h")]
    return max(os.path.getmtime(h) for h in hdrs)


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(
            os.path.getmtime(src), _deps()):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
