"""Alpha-compositing path (the north star's secondary path, reference
rasterize.py:14-253 / forward.cu:252-374 / backward.cu:138-315) at 1080p:
project_gaussians_2d + rasterize_gaussians forward, and forward + backward,
per call through the drop-in operator API.  Run under
``rocprofv3 --kernel-trace --stats`` for the raster_alpha kernels' times.

    python tools/alphabench.py [--splats 10000 50000] [--calls 200]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# A/B knobs and timestamped variants: the diagnostic library (gsvc_amd/_lib.py)
os.environ.setdefault("GSVC_DIAG", "1")

import torch  # noqa: E402

H, W = 1080, 1920


def run(n, calls, dev, backward):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize import rasterize_gaussians
    g = torch.Generator().manual_seed(n)
    means = torch.tanh(torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5))).to(dev).requires_grad_(backward)
    L = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5])).to(dev).requires_grad_(backward)
    col = torch.rand(n, 3, generator=g).to(dev).requires_grad_(backward)
    opac = (0.1 + 0.9 * torch.rand(n, 1, generator=g)).to(dev).requires_grad_(backward)
    bg = torch.ones(3, device=dev)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)

    def step():
        xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
        out = rasterize_gaussians(xys, depths, radii, conics, nth, col, opac, H, W, 16, 16,
                                  background=bg)
        if backward:
            out.sum().backward()
        return out

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(calls):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / calls * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, nargs="+", default=[10000, 50000])
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--knob", action="append", default=[],
                    help="K=V: gsvc_debug_set(K, V) first (A/B; knob 9 = 1: shuffle reductions)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.knob:
        from gsvc_amd import _lib as L
        lib = L.load()
        for kv in a.knob:
            k, v = kv.split("=")
            if lib.gsvc_debug_set(int(k), int(v)) < 0:
                raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")
    for n in a.splats:
        fwd = run(n, a.calls, dev, False)
        both = run(n, a.calls, dev, True)
        print(json.dumps(dict(path="rasterize_gaussians (alpha)", H=H, W=W, splats=n,
                              us_forward=round(fwd, 1), us_forward_backward=round(both, 1), knobs=a.knob)),
              flush=True)


if __name__ == "__main__":
    main()
