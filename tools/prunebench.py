"""Prune cost: gsvc_prune_lowest vs the reference's torch sequence (norm, sort,
boolean mask, four p[keep]) on the GPU, for a 100k-splat frame model.

    python tools/prunebench.py [--splats 100000] [--remove 250 10000] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gsvc_amd.prune import prune_lowest  # noqa: E402


def torch_prune(ps, k):
    rgb_weight = torch.norm(ps[3], dim=1)
    _, order = torch.sort(rgb_weight)
    keep = torch.ones(ps[0].shape[0], dtype=torch.bool, device=ps[0].device)
    keep[order[:k]] = False
    return [p[keep] for p in ps]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, default=100000)
    ap.add_argument("--remove", type=int, nargs="+", default=[250, 10000])
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    n = a.splats
    ps = [torch.rand(n, c, generator=g).to(dev) for c in (2, 3, 3)]
    w = torch.rand(n, 1, generator=g)
    w[: n // 10] = 0.01  # a densified block: one tie group
    ps.append(w.to(dev))
    for k in a.remove:
        res = {}
        for name, fn in (("kernel", lambda: prune_lowest(ps[3], ps, k)),
                         ("torch", lambda: torch_prune(ps, k))):
            for _ in range(5):
                out = fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                out = fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = (e0.elapsed_time(e1) * 1e3 / a.iters, out)
        same = all(torch.equal(x, y) for x, y in zip(res["kernel"][1], res["torch"][1]))
        print(json.dumps(dict(splats=n, remove=k, kernel_us=round(res["kernel"][0], 1),
                              torch_us=round(res["torch"][0], 1), identical=same)), flush=True)


if __name__ == "__main__":
    main()
