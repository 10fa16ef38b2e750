"""Microbenchmark of the composite kernels (rasterize_sum forward/backward).

    python tests/analysis/kbench.py [--splats 10000 50000] [--variants 0 1] [--iters 200]

Sets up a 1920x1080 frame (reference init distributions), bins it, then for
each kernel variant (C-ABI knob gsvc_debug_set(0, v); 0 = automatic) captures ``iters``
back-to-back launches in a HIP graph and replays it, so host launch overhead
cannot starve the GPU; prints average microseconds per launch and the
algorithmic-bytes rate.  Outputs of every variant are checked bit-identical to
variant 0.  Run it under ``rocprofv3 --kernel-trace --stats`` for per-dispatch
durations and under ``--pmc`` for counters.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
# A/B knobs and timestamped variants: the diagnostic library (gsvc_amd/_lib.py)
os.environ.setdefault("GSVC_DIAG", "1")

import torch  # noqa: E402

from gsvc_amd import _lib as L  # noqa: E402
from gsvc_amd import ops  # noqa: E402

H, W = 1080, 1920


def setup(n, seed, chol_scale=1.0):
    import oracle as O
    means, chol, colors, opac = O.synthetic_frame(n, seed, chol_scale=chol_scale)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(chol), H, W, tb, 0.01)
    from gsvc_amd.utils import bin_and_sort_for_raster
    m, gids, bins = bin_and_sort_for_raster(n, xys, depths, radii, nth, tb)
    counts = (bins[:, 1] - bins[:, 0]).clamp(min=0, max=256)
    shape = dict(N=n, N_vis=int((nth > 0).sum()), M=m, M_eff=int(counts.sum()),
                 max_per_tile=int((bins[:, 1] - bins[:, 0]).max()), T=tb[0] * tb[1], P=H * W)
    return dict(tb=tb, xys=xys, conics=conics, colors=T(colors), opac=T(opac), gids=gids, bins=bins,
                bg=torch.ones(3, device=dev), shape=shape, dev=dev)


def fwd_args(s, out, idx, layout=0):
    tb = s["tb"]
    return (tb[0], tb[1], 1, 16, 16, 1, W, H, 1, L.ptr(s["gids"]), L.ptr(s["bins"]), L.ptr(s["xys"]),
            L.ptr(s["conics"]), L.ptr(s["colors"]), L.ptr(s["opac"]), L.ptr(s["bg"]), None,
            s["shape"]["M"], layout, L.ptr(out), None, L.ptr(idx), L.stream(s["dev"]))


def bwd_args(s, idx, v_out, rec):
    n = s["xys"].shape[0]
    return (H, W, 16, 16, n, L.ptr(s["gids"]), L.ptr(s["bins"]), L.ptr(s["xys"]), L.ptr(s["conics"]),
            L.ptr(s["colors"]), L.ptr(s["opac"]), L.ptr(s["bg"]), None, L.ptr(idx), L.ptr(v_out),
            None, L.ptr(rec), L.stream(s["dev"]))


def time_graph(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, nargs="+", default=[10000, 50000])
    ap.add_argument("--variants", type=int, nargs="+", default=[0])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--chol-scale", type=float, default=1.0)
    ap.add_argument("--backward", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="run the timestamp build (mode 3)")
    ap.add_argument("--thresholds", type=int, nargs="*", default=[],
                    help="per-tile thresholds to sweep for mode 6 (variant id 1000 + t)")
    args = ap.parse_args()
    lib = L.load()
    results = []
    for n in args.splats:
        s = setup(n, seed=n, chol_scale=args.chol_scale)
        sh = s["shape"]
        nbytes = 36 * sh["N_vis"] + 4 * sh["M_eff"] + 8 * sh["T"] + 16 * sh["P"]
        ref_out = ref_idx = None
        lib.gsvc_debug_set(1, n)  # splat count for the packed-record experiment
        for v in list(args.variants) + [1000 + t for t in args.thresholds]:
            lib.gsvc_debug_set(0, v if v < 1000 else 6)
            lib.gsvc_debug_set(3, v - 1000 if v >= 1000 else 0)
            out = torch.empty((H, W, 3), device=s["dev"])
            idx = torch.empty((H, W), dtype=torch.int32, device=s["dev"])
            us = time_graph(lambda: L.call("gsvc_rasterize_sum_forward_ex", *fwd_args(s, out, idx)),
                            args.iters)
            if ref_out is None:
                ref_out, ref_idx = out.clone(), idx.clone()
                same = True
            else:
                same = bool(torch.equal(out, ref_out) and torch.equal(idx, ref_idx))
            rec = dict(kernel="sum_fwd", variant=v, us=round(us, 2),
                       GBs=round(nbytes / us / 1e3, 1), frac=round(nbytes / us / 1e3 / 8000, 4),
                       identical=same, **sh)
            results.append(rec)
            print(json.dumps(rec), flush=True)
        if args.stamps:
            lib.gsvc_debug_set(0, 3)
            out = torch.empty((H, W, 3), device=s["dev"])
            idx = torch.empty((H, W), dtype=torch.int32, device=s["dev"])
            st = torch.zeros((s["shape"]["T"], 4), dtype=torch.int64, device=s["dev"])
            a = list(fwd_args(s, out, idx))
            a[20] = L.ptr(st)
            for _ in range(3):
                L.call("gsvc_rasterize_sum_forward_ex", *a)
            torch.cuda.synchronize()
            t = st.cpu().numpy().astype(np.float64)
            t0 = t[:, 0].min()
            us = lambda x: (x - t0) * 10.0 / 1000.0  # 100 MHz ticks -> us  # noqa: E731
            q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa: E731
            w1 = t[:, 2] > 0
            rec = dict(kernel="sum_fwd_stamps", N=n, wave0_start=q(us(t[:, 0])),
                       wave0_dur=q(t[:, 1] * 0.01 - t[:, 0] * 0.01), wave0_end=q(us(t[:, 1])),
                       dense_tiles=int(w1.sum()),
                       wave1_dur=q((t[w1, 3] - t[w1, 2]) * 0.01) if w1.any() else None)
            print(json.dumps(rec), flush=True)
            lib.gsvc_debug_set(0, 0)
        if args.backward:
            lib.gsvc_debug_set(0, 0)
            out = torch.empty((H, W, 3), device=s["dev"])
            idx = torch.empty((H, W), dtype=torch.int32, device=s["dev"])
            L.call("gsvc_rasterize_sum_forward_ex", *fwd_args(s, out, idx))
            v_out = torch.randn((H, W, 3), device=s["dev"])
            rec_t = torch.empty((n, 16), device=s["dev"])
            us = time_graph(lambda: L.call("gsvc_rasterize_sum_backward",
                                           *bwd_args(s, idx, v_out, rec_t)), args.iters)
            bb = 16 * sh["P"] + 36 * sh["N_vis"] + 4 * sh["M_eff"] + 8 * sh["T"] + 36 * n
            r = dict(kernel="sum_bwd", us=round(us, 2), GBs=round(bb / us / 1e3, 1),
                     frac=round(bb / us / 1e3 / 8000, 4), **sh)
            results.append(r)
            print(json.dumps(r), flush=True)
    lib.gsvc_debug_set(0, 0)
    lib.gsvc_debug_set(3, 0)


if __name__ == "__main__":
    main()
