"""Build recipe for the gfx950 C-ABI libraries.

    python -m gsvc_amd.build            # or __graft_entry__.build()

``gsvc_amd/lib/libgsvc_amd.so`` is the product library (include/gsvc_amd.h);
``gsvc_amd/lib/libgsvc_amd_diag.so`` the diagnostic one, the same sources with
``-DGSVC_DIAG``: A/B knobs, timestamped and ablation kernel variants
(include/gsvc_amd_diag.h), for tools/ and the variant-comparison tests only.
One ``hipcc --offload-arch=gfx950`` compile per ``.hip`` source and variant
(object files cached under gsvc_amd/lib/obj* by mtime), then one shared-object
link each.  The libraries are built in-tree so they travel to the GPU box with
the repo snapshot.  ``-ffp-contract=off`` fixes the floating-point op sequence
(every fused multiply-add in the kernels is an explicit ``fmaf``), which the
CPU oracle restates; see DESIGN.md §4.
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
LIB = os.path.join(LIBDIR, "libgsvc_amd.so")
LIB_DIAG = os.path.join(LIBDIR, "libgsvc_amd_diag.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC", "-std=c++17",
         "-Wall", "-Wno-unused-result"]
VARIANTS = {LIB: ("obj", []), LIB_DIAG: ("obj_diag", ["-DGSVC_DIAG"])}
# the C++ autograd Functions of the drop-in operators (csrc/torch_ops.cpp),
# a torch extension module linked against the product library
TORCH_EXT = os.path.join(LIBDIR, "_torch_ops.so")
# the CPU dispatch of the two operators (csrc/cpu_ops.cpp): host code only
CPU_LIB = os.path.join(LIBDIR, "libgsvc_amd_cpu.so")
CPU_SRC = os.path.join(CSRC, "cpu_ops.cpp")
TORCH_EXT_SRC = os.path.join(CSRC, "torch_ops.cpp")


def _deps():
    inc = os.path.join(os.path.dirname(HERE), "include")
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(inc, "*.h"))
    return max(os.path.getmtime(h) for h in hdrs)


def _compile(src: str, objdir: str, defs, force: bool) -> str:
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(
            os.path.getmtime(src), _deps()):
        return obj
    cmd = [HIPCC, *FLAGS, *defs, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs = []
    for lib, (sub, defs) in VARIANTS.items():
        objdir = os.path.join(LIBDIR, sub)
        os.makedirs(objdir, exist_ok=True)
        jobs += [(lib, s, objdir, defs) for s in srcs]
    with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        objs = list(ex.map(lambda j: (j[0], _compile(j[1], j[2], j[3], force)), jobs))
    for lib in VARIANTS:
        mine = [o for l, o in objs if l == lib]
        if force or not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in mine):
            tmp = lib + ".tmp"
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC",
                   f"-Wl,-soname,{os.path.basename(lib)}", "-o", tmp, *mine]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
            os.replace(tmp, lib)
        if verbose:
            print(lib)
    _build_torch_ext(force, verbose)
    _build_cpu_lib(force, verbose)
    return LIB


def _build_cpu_lib(force: bool, verbose: bool) -> None:
    """g++ with OpenMP, -ffp-contract=off and no fast math (the kernels' op
    sequence)."""
    if not force and os.path.exists(CPU_LIB) and os.path.getmtime(CPU_LIB) >= os.path.getmtime(CPU_SRC):
        if verbose:
            print(CPU_LIB)
        return
    tmp = CPU_LIB + ".tmp"
    cmd = ["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
           "-fopenmp", "-Wall", CPU_SRC, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"CPU library build failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, CPU_LIB)
    if verbose:
        print(CPU_LIB)


def _build_torch_ext(force: bool, verbose: bool) -> None:
    """hipcc (host C++ only) against torch's headers and libraries, with an
    rpath to this directory for libgsvc_amd.so."""
    if (not force and os.path.exists(TORCH_EXT) and os.path.getmtime(TORCH_EXT) >= max(
            os.path.getmtime(TORCH_EXT_SRC), os.path.getmtime(LIB), _deps())):
        if verbose:
            print(TORCH_EXT)
        return
    import sysconfig

    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           sysconfig.get_paths()["include"]]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tmp = TORCH_EXT + ".tmp"
    cmd = [HIPCC, "-O2", "-fPIC", "-shared", "-std=c++17", "-w",
           "-DTORCH_EXTENSION_NAME=_torch_ops", "-DTORCH_API_INCLUDE_EXTENSION_H",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           *[f"-I{d}" for d in inc], TORCH_EXT_SRC,
           f"-L{os.path.join(tdir, 'lib')}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
           "-ltorch_hip", "-ltorch_python", f"-L{LIBDIR}", "-lgsvc_amd",
           "-Wl,-rpath,$ORIGIN", "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch extension build failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, TORCH_EXT)
    if verbose:
        print(TORCH_EXT)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
