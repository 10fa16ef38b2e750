"""Disassemble the gfx950 code of a built object or library, optionally one
kernel only, and count its instructions by class (VALU / SALU / LDS / VMEM /
SMEM / branch) -- a static cross-check for the SQ_INSTS_* counters.

    python tools/isa_dump.py gsvc_amd/lib/obj/raster_sum.hip.o --kernel 'raster_sum_fwd_kernelILi9ELb0E' [--out f.s]
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from store_hazard_scan import LLVM, code_objects  # noqa: E402


def classify(mn: str) -> str:
    if mn.startswith(("ds_",)):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith("s_load") or mn.startswith("s_buffer_load") or mn.startswith("s_memrealtime"):
        return "smem"
    if mn.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if mn.startswith("s_waitcnt") or mn.startswith("s_nop") or mn.startswith("s_barrier"):
        return "wait"
    if mn.startswith("s_"):
        return "salu"
    if mn.startswith("v_"):
        return "valu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default=None, help="substring of the mangled kernel name")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        text = ""
        for co in code_objects(a.path, tmp):
            r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950",
                                "--no-show-raw-insn", co], capture_output=True, text=True)
            text += r.stdout
    blocks = re.split(r"\n(?=[0-9a-f]+ <[^>]+>:)", text)
    sel = [b for b in blocks if a.kernel is None or (b.split("\n", 1)[0].find(a.kernel) >= 0)]
    out = "\n".join(sel)
    if a.out:
        open(a.out, "w").write(out)
    for b in sel:
        head = b.split("\n", 1)[0]
        cnt = collections.Counter()
        for line in b.split("\n")[1:]:
            s = line.strip()
            if not s or s.startswith(";") or s.endswith(":"):
                continue
            parts = s.split()
            mn = parts[0] if not re.match(r"^[0-9a-f]+$", parts[0]) else (parts[1] if len(parts) > 1 else "")
            cnt[classify(mn)] += 1
        if sum(cnt.values()) > 20:
            print(head[:120], dict(cnt))


if __name__ == "__main__":
    main()
