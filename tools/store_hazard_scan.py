"""Static check of the gfx950 store-data hazard in a built library.

A vector-memory store of more than 64 bits of data (``*_store_dwordx3/x4``)
reads its data VGPRs after it issues; on gfx940+ a VALU instruction that
overwrites one of those VGPRs needs at least TWO wait states after the store
(one on earlier gfx9).  The compiler inserts them for the stores it generates
and, in straight-line code, for inline-asm stores too -- but round 5's HWC
write-through store (``global_store_dwordx4 ... sc1 nt`` as inline asm at the
end of an exec-masked block) was followed across the block boundary by
``s_or_b64 exec`` (one wait state) and a ``v_or_b32`` into the first data VGPR:
the store then wrote the new value for one 16-lane pass of the wave now and
then.

This scanner disassembles every gfx950 code object of a library / object file
and walks each >64-bit store's successors (fall-through and branch targets)
until two wait states have passed, reporting any VALU write to a data VGPR
inside that window.  ``s_nop N`` counts N + 1 wait states, every other
instruction one.

    python tools/store_hazard_scan.py gsvc_amd/lib/libgsvc_amd.so [...]

Exit status 1 when a hazard is found.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = os.environ.get("GSVC_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
WAIT_STATES = 2  # gfx940+ (LLVM GCNHazardRecognizer::checkVALUHazardsHelper)

_INSN = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):")
_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def _vregs(op: str):
    m = _VREG.match(op.strip())
    if not m:
        return None
    if m.group(1) is not None:
        r = int(m.group(1))
        return r, r
    return int(m.group(2)), int(m.group(3))


def _store_data(mn: str, ops):
    """VGPR range of a >64-bit VMEM store's data operand, else None."""
    if not re.match(r"^(global|flat|scratch|buffer)_store_(dwordx[34]|b96|b128)$", mn):
        return None
    idx = 0 if mn.startswith("buffer_") else 1
    return _vregs(ops[idx]) if len(ops) > idx else None


def _valu_vdst(mn: str, ops):
    if not mn.startswith("v_") or not ops:
        return None
    return _vregs(ops[0])


def _waits(mn: str, ops) -> int:
    if mn == "s_nop":
        return int(ops[0], 0) + 1
    return 1


def code_objects(path: str, tmp: str):
    """gfx950 code objects inside a shared library / object (.hip_fatbin)."""
    objcopy = os.path.join(LLVM, "llvm-objcopy")
    bundler = os.path.join(LLVM, "clang-offload-bundler")
    fat = os.path.join(tmp, os.path.basename(path) + ".fatbin")
    r = subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", path, os.devnull],
                       capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(fat):
        raise RuntimeError(f"no .hip_fatbin in {path}: {r.stderr.strip()}")
    # a linked library holds one bundle per translation unit, back to back
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        part = os.path.join(tmp, f"b{i}.bundle")
        with open(part, "wb") as f:
            f.write(data[s:e])
        co = os.path.join(tmp, f"b{i}.co")
        r = subprocess.run([bundler, "--unbundle", "--type=o", f"--targets={TARGET}",
                            f"--input={part}", f"--output={co}"], capture_output=True, text=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    if not out:
        raise RuntimeError(f"no {TARGET} code object in {path}")
    return out


def parse(disasm: str):
    """{function: [(addr, mnemonic, operands)]}"""
    funcs, cur = {}, None
    for line in disasm.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            ops = [o.strip() for o in m.group(2).split(",")] if m.group(2) else []
            cur.append((int(m.group(3), 16), m.group(1), ops))
    return funcs


def scan_function(insns):
    at = {a: i for i, (a, _, _) in enumerate(insns)}
    found = []
    for i, (addr, mn, ops) in enumerate(insns):
        data = _store_data(mn, ops)
        if data is None:
            continue
        lo, hi = data
        # DFS over (index, wait states so far)
        stack, seen = [(i + 1, 0)], set()
        while stack:
            j, w = stack.pop()
            if j >= len(insns) or w >= WAIT_STATES or (j, w) in seen:
                continue
            seen.add((j, w))
            a2, mn2, ops2 = insns[j]
            d = _valu_vdst(mn2, ops2)
            if d is not None and d[0] <= hi and lo <= d[1]:
                found.append((addr, mn, ops, a2, mn2, ops2, w))
                continue
            if mn2 == "s_endpgm" or mn2.startswith("s_setpc") or mn2.startswith("s_trap"):
                continue
            w2 = w + _waits(mn2, ops2)
            if mn2 == "s_branch" or mn2.startswith("s_cbranch"):
                tgt = a2 + 4 + 4 * int(ops2[0], 0)
                if tgt in at:
                    stack.append((at[tgt], w2))
                if mn2 == "s_branch":
                    continue
            stack.append((j + 1, w2))
    return found


def scan(path: str):
    objdump = os.path.join(LLVM, "llvm-objdump")
    hits = []
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(path, tmp):
            r = subprocess.run([objdump, "-d", "--mcpu=gfx950", co], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(r.stderr)
            for fn, insns in parse(r.stdout).items():
                for h in scan_function(insns):
                    hits.append((fn,) + h)
    return hits


def main(argv):
    bad = 0
    for path in argv or [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "gsvc_amd", "lib", "libgsvc_amd.so")]:
        hits = scan(path)
        print(f"{path}: {len(hits)} store-data hazard(s)")
        for fn, a, mn, ops, a2, mn2, ops2, w in hits:
            print(f"  {fn}\n    {a:#x} {mn} {', '.join(ops)}\n    {a2:#x} {mn2} {', '.join(ops2)}"
                  f"   <- {w} wait state(s)")
        bad += len(hits)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
