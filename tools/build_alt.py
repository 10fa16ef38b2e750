"""Build the diagnostic library of another version of the kernel sources as an
A/B variant: gsvc_amd/lib/alt/<name>/libgsvc_amd_diag.so, for
tools/ab_builds.sh (which runs every variant interleaved).

    python tools/build_alt.py NAME [--ref GIT_REF]      # the sources at a commit
    python tools/build_alt.py NAME --define -DFOO=1      # the working tree + defines
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gsvc_amd import build as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--ref", default=None, help="git ref of gsvc_amd/csrc and include/ (default: working tree)")
    ap.add_argument("--define", action="append", default=[])
    ap.add_argument("--product", action="store_true",
                    help="the product library (no -DGSVC_DIAG) as alt/NAME/libgsvc_amd.so, for "
                         "tools/ab_product.sh (bench.py with the library swapped)")
    a = ap.parse_args()
    out = os.path.join(REPO, "gsvc_amd", "lib", "alt", a.name)
    os.makedirs(out, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "src")
        if a.ref:
            os.makedirs(src)
            tar = subprocess.run(["git", "-C", REPO, "archive", a.ref, "gsvc_amd/csrc", "include"],
                                 check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", src], input=tar, check=True)
        else:
            shutil.copytree(os.path.join(REPO, "gsvc_amd", "csrc"), os.path.join(src, "gsvc_amd", "csrc"))
            shutil.copytree(os.path.join(REPO, "include"), os.path.join(src, "include"))
        csrc = os.path.join(src, "gsvc_amd", "csrc")
        objs = []
        for f in sorted(glob.glob(os.path.join(csrc, "*.hip"))):
            o = os.path.join(tmp, os.path.basename(f) + ".o")
            cmd = [B.HIPCC, *B.FLAGS, *([] if a.product else ["-DGSVC_DIAG"]), *a.define, f"-I{os.path.join(src, 'include')}",
                   "-c", f, "-o", o]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                sys.exit(f"hipcc failed for {f}:\n{r.stderr}")
            objs.append(o)
        name = "libgsvc_amd.so" if a.product else "libgsvc_amd_diag.so"
        lib = os.path.join(out, name)
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC",
                        f"-Wl,-soname,{name}", "-o", lib, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
