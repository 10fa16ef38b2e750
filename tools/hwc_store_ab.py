"""A/B of the op path's HWC row stores: plain (the product) vs padded
write-through (``sc1 nt`` + ``s_nop 1``, the render planes' policy), now that
round 5's loss is explained.  Renders seeded 1080p frames
through the Python Function (counted binning + rasterize_sum_forward_ex, the
``raster_sum_fwd_kernel<1, true>`` composite) on the library GSVC_DIAG_LIB
names; run it under rocprofv3 once per library and compare that kernel's
average duration:

    GSVC_DIAG=1 GSVC_DIAG_LIB=gsvc_amd/lib/libgsvc_amd_diag.so python tools/hwc_store_ab.py
    GSVC_DIAG=1 GSVC_DIAG_LIB=gsvc_amd/lib/repro/libgsvc_amd_r5hwc_nop.so python tools/hwc_store_ab.py

(the second library is tests/analysis/store_hazard_repro.py --build's padded form).
Prints the HIP-event time per forward and a checksum of the image.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("GSVC_DIAG", "1")

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, nargs="+", default=[10000, 50000])
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    for n in a.splats:
        g = torch.Generator().manual_seed(n)
        means = (2 * torch.rand(n, 2, generator=g) - 1).to(dev)
        L = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5])).to(dev)
        col = torch.rand(n, 3, generator=g).to(dev)
        o = torch.ones(n, 1, device=dev)
        bg = torch.ones(3, device=dev)
        xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
        for _ in range(10):
            img = rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, o, H, W, 16, 16, background=bg)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            img = rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, o, H, W, 16, 16, background=bg)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"lib": os.path.basename(os.environ.get("GSVC_DIAG_LIB", "diag")), "n": n,
                          "us_per_forward": e0.elapsed_time(e1) * 1000 / a.iters,
                          "checksum": float(img.double().sum())}), flush=True)


if __name__ == "__main__":
    main()
