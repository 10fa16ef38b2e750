"""Microbenchmark of the one-call frame render (gsvc_render_frame_sum).

    python tools/fbench.py [--splats 10000 50000] [--iters 200] [--chol-scale 1]

For each rasterizer mode (gsvc_debug_set(0)) captures ``iters`` back-to-back
frame renders in a HIP graph, replays it and prints microseconds per frame.
Every mode's image must equal the first one bit for bit.  (A frame inside a
graph keeps its frame_index argument from capture time; the two M slots then
alternate only between replays, so frames of one replay share a slot --
harmless here since every frame renders the same splats.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from gsvc_amd import _lib as L  # noqa: E402

H, W = 1080, 1920


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, nargs="+", default=[10000, 50000])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--chol-scale", type=float, default=1.0)
    ap.add_argument("--modes", type=int, nargs="+", default=[0],
                    help="rasterizer modes (gsvc_debug_set(0)); 0 = automatic")
    args = ap.parse_args()
    lib = L.load()
    dev = torch.device("cuda:0")
    for n in args.splats:
        g = torch.Generator().manual_seed(n)
        xyz = torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5)).to(dev)
        chol = (torch.rand(n, 3, generator=g) * args.chol_scale).to(dev)
        feat = torch.rand(n, 3, generator=g).to(dev)
        bound = torch.tensor([0.5, 0.0, 0.5], device=dev)
        bg = torch.ones(3, device=dev)
        ws_bytes = L.size("gsvc_render_frame_workspace_bytes", n, H, W)
        ws = torch.zeros((ws_bytes,), dtype=torch.uint8, device=dev)
        meta = torch.zeros((2,), dtype=torch.int32, device=dev)
        out = torch.empty((1, 3, H, W), device=dev)
        ref = None
        counter = [0]
        for mode in args.modes:
            lib.gsvc_debug_set(0, mode)

            def frame():
                L.call("gsvc_render_frame_sum", n, L.ptr(xyz), 1, L.ptr(chol), L.ptr(bound),
                       L.ptr(feat), None, None, L.ptr(bg), H, W, counter[0], 0, L.ptr(meta),
                       L.ptr(ws), ws_bytes, L.ptr(out), L.stream(dev))
                counter[0] += 1

            frame()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(args.iters):
                    frame()
            gr.replay()
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(3):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                gr.replay()
                b.record()
                torch.cuda.synchronize()
                best = min(best, a.elapsed_time(b) * 1e3 / args.iters)
            same = True
            if ref is None:
                ref = out.clone()
            else:
                same = bool(torch.equal(out, ref))
            m = int(meta[0])
            print(json.dumps(dict(N=n, M=m, mode=mode,
                                  us_per_frame=round(best, 2), fps=round(1e6 / best, 0),
                                  identical=same)), flush=True)
    lib.gsvc_debug_set(0, 0)


if __name__ == "__main__":
    main()
