"""Host cost of the drop-in operator path (what GSVC's own, unchanged
GaussianSplats_Represent.py runs): project_gaussians_2d + rasterize_gaussians_sum
forward and backward on a tiny frame (no GPU back-pressure), per call, and the
same ops at 1080p / 50k (GPU-bound) for scale.

    python tools/opbench.py [--calls 500]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def run(n, H, W, calls, dev, backward):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    g = torch.Generator().manual_seed(0)
    means = torch.tanh(torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5))).to(dev).requires_grad_(backward)
    L = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5])).to(dev).requires_grad_(backward)
    col = torch.rand(n, 3, generator=g).to(dev).requires_grad_(backward)
    opac = torch.ones(n, 1, device=dev)
    bg = torch.ones(3, device=dev)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)

    def step():
        xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, opac, H, W, 16, 16,
                                      background=bg)
        if backward:
            out.sum().backward()
        return out

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    for _ in range(calls):
        step()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / calls * 1e6
    return us, (torch.cuda.max_memory_allocated(dev) - base) / 2**20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=500)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {}
    for bw in (False, True):
        tag = "fwd_bwd" if bw else "fwd"
        us, _ = run(16, 16, 16, a.calls, dev, bw)
        res[f"tiny_{tag}_us"] = round(us, 1)
        us, mib = run(50000, 1080, 1920, a.calls // 5, dev, bw)
        res[f"1080p_50k_{tag}_us"] = round(us, 1)
        res[f"1080p_50k_{tag}_peak_extra_MiB"] = round(mib, 1)
    res["note"] = ("unchanged-caller path: gsplat.project_gaussians_2d + rasterize_gaussians_sum "
                   "(+ .sum().backward()); peak_extra = max_memory_allocated above the "
                   "resident inputs during the timed calls")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
