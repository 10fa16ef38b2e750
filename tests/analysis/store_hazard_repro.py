"""Reproduction of round 5's lost-row store fault and of its cause.

Round 5 wrote the op path's HWC image with inline-asm write-through stores
(``global_store_dwordx4 ... sc1 nt``) and 68-288 random tiles per 1080p frame
came out wrong, 16 pixels each (profiles/r05/op_path/mm*.log).  Hypothesis:
the gfx940+ VALU-after-store data hazard -- in that build the first of the
three row stores ended an exec-masked block, and the next block's first VALU
(``v_or_b32 vD, 64, lane``: the next chunk index) overwrote the store's first
data VGPR one wait state after it, where two are needed.

Predictions (written before the GPU run):
  * wrong values only at tile-local HWC float offsets 4c with c in 0..63 (the
    first row store's chunks, data VGPR 0 = the chunk's first float), and
    within a tile only the chunks of ONE 16-lane pass: 16 floats -> 16 pixels;
  * the wrong float's bits are the integer 64 + c (the overwriting value);
  * the same source with ``s_nop 1`` after the asm store (the fix) renders
    bit-identically to the product library.

Result (profiles/r06/store_hazard/repro_gpu.log, 4 calls each at 50k and 9k):
the bare build lost 48-65 tiles per call at 50k and 252-328 at 9k, always 16
floats per tile, always at offset 4c (data VGPR 0), and the wrong bits equal
64 + c in every case; the padded build: 0 differing floats in all 8 calls.
The lane prediction was off in its detail: the 16 lanes are the LAST QUAD of
each 16-lane row (c mod 16 in 12..15, one quad per row), not one 16-lane pass.

``--build`` (CPU, this container): writes the round-5 HWC form of
raster_sum.hip into gsvc_amd/lib/repro/ (the current source with the HWC row
store replaced by the bare asm store, or the padded one with ``--padded``),
compiles it with the product flags, links it with the diagnostic objects into
``libgsvc_amd_r5hwc.so`` / ``libgsvc_amd_r5hwc_nop.so`` (used as
GSVC_DIAG_LIB: the Python Function's forward then runs its kernels), and runs
tools/store_hazard_scan.py on both.

GPU: ``python tests/analysis/store_hazard_repro.py --run [--repeat 4]``
renders seeded 1080p frames through the Python Function on each library and on
the product library, and reports every differing float.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
LIBDIR = os.path.join(REPO, "gsvc_amd", "lib")
OUT = os.path.join(LIBDIR, "repro")
VARIANTS = {"r5hwc": "bare", "r5hwc_nop": "padded"}

_HWC_NOW = re.compile(r"                const float4 q = s_slice\[c\];\n                st_f4\(o, q\.x, q\.y, q\.z, q\.w, A\.store_policy\);\n")


def _variant_source(form: str) -> str:
    src = open(os.path.join(REPO, "gsvc_amd", "csrc", "raster_sum.hip")).read()
    m = _HWC_NOW.search(src)
    assert m, "HWC store block not found in raster_sum.hip"
    nop = "\\n\\ts_nop 1" if form == "padded" else ""
    body = ("                const float4 q = s_slice[c];\n"
            "                const v4f v = {q.x, q.y, q.z, q.w};\n"
            f"                asm volatile(\"global_store_dwordx4 %0, %1, off sc1 nt{nop}\" "
            "::\"v\"(o), \"v\"(v) : \"memory\");\n")
    return src[:m.start()] + body + src[m.end():]


def build():
    from gsvc_amd import build as B
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import store_hazard_scan as S
    B.build()
    os.makedirs(OUT, exist_ok=True)
    diag_objs = [os.path.join(LIBDIR, "obj_diag", f) for f in sorted(os.listdir(os.path.join(LIBDIR, "obj_diag")))
                 if f.endswith(".o") and f != "raster_sum.hip.o"]
    for name, form in VARIANTS.items():
        # the source sits in csrc's directory so its relative includes resolve
        src = os.path.join(REPO, "gsvc_amd", "csrc", f"_repro_{name}.hip")
        obj = os.path.join(OUT, f"raster_sum_{name}.o")
        lib = os.path.join(OUT, f"libgsvc_amd_{name}.so")
        with open(src, "w") as f:
            f.write(_variant_source(form))
        try:
            subprocess.run([B.HIPCC, *B.FLAGS, "-c", src, "-o", obj], check=True, capture_output=True)
        finally:
            os.remove(src)
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, obj, *diag_objs],
                       check=True, capture_output=True)
        hits = S.scan(obj)
        print(json.dumps({"variant": name, "form": form, "lib": os.path.relpath(lib, REPO),
                          "hazards": [{"kernel": h[0], "store": f"{h[2]} {', '.join(h[3])}",
                                       "valu": f"{h[5]} {', '.join(h[6])}", "wait_states": h[7]}
                                      for h in hits]}))
    print(json.dumps({"product": "gsvc_amd/lib/libgsvc_amd.so",
                      "hazards": len(S.scan(os.path.join(LIBDIR, "libgsvc_amd.so")))}))


def _frame(n, H, W, dev, seed):
    import torch
    g = torch.Generator().manual_seed(seed)
    means = (2 * torch.rand(n, 2, generator=g) - 1).to(dev)
    L = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5])).to(dev)
    col = torch.rand(n, 3, generator=g).to(dev)
    return means, L, col


def _render(means, L, col, H, W):
    import torch
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    o = torch.ones(means.shape[0], 1, device=means.device)
    bg = torch.ones(3, device=means.device)
    xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
    return rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, o, H, W, 16, 16, background=bg)


def run(repeat: int):
    import torch
    from gsvc_amd import _lib
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    tbx = (W + 15) // 16
    cases = [(50000, 51080), (9000, 10080)]
    for n, seed in cases:
        means, L, col = _frame(n, H, W, dev, seed)
        # reference: the product library's Python Function (plain HWC stores)
        _lib._active = _lib._open(_lib.LIB_PATH, False)
        ref = _render(means, L, col, H, W).detach().contiguous()
        torch.cuda.synchronize()
        for name in VARIANTS:
            lib = _lib._open(os.path.join(OUT, f"libgsvc_amd_{name}.so"), True)
            _lib._active = lib
            for r in range(repeat):
                img = _render(means, L, col, H, W).detach().contiguous()
                torch.cuda.synchronize()
                bad = (img != ref)
                nbad = int(bad.sum())
                rec = {"n": n, "variant": name, "rep": r, "bad_floats": nbad}
                if nbad:
                    ys, xs, ch = torch.nonzero(bad, as_tuple=True)
                    tiles = (ys // 16) * tbx + xs // 16
                    # tile-local HWC float offset and 16-byte chunk (one lane each)
                    off = ((ys % 16) * 16 + xs % 16) * 3 + ch
                    chunk = off // 4
                    bits = img[ys, xs, ch].view(torch.int32)
                    ut = torch.unique(tiles)
                    per_tile = torch.bincount(torch.searchsorted(ut, tiles))
                    passes = torch.unique(chunk // 16)
                    rec.update({
                        "bad_tiles": int(ut.numel()),
                        "bad_floats_per_tile": sorted(set(per_tile.tolist())),
                        "offset_mod_4": sorted(set((off % 4).tolist())),
                        "chunk_min": int(chunk.min()), "chunk_max": int(chunk.max()),
                        "lane_passes": passes.tolist(),
                        "lanes_mod_16": sorted(set((chunk % 16).tolist())),
                        "bits_equal_64_plus_chunk": bool((bits == 64 + chunk).all()),
                        "bits_sample": bits[:8].tolist(), "chunk_sample": chunk[:8].tolist(),
                        "maxdiff": float((img - ref).abs().max()),
                    })
                print(json.dumps(rec), flush=True)
        _lib._active = None


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--repeat", type=int, default=4)
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.repeat)
