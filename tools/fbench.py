"""Microbenchmark of the one-call frame render (gsvc_render_frame_sum).

    python tools/fbench.py [--splats 10000 50000] [--iters 200] [--chol-scale 1]

For each rasterizer mode (gsvc_debug_set(0)) and each extra knob pass, times
``iters`` back-to-back frame renders (plain library calls; the slab entries
refuse graph capture since round 5) and prints microseconds per frame, best
of three.  Every pass's image must equal the first one bit for bit.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# A/B knobs and timestamped variants: the diagnostic library (gsvc_amd/_lib.py)
os.environ.setdefault("GSVC_DIAG", "1")

import torch  # noqa: E402

from gsvc_amd import _lib as L  # noqa: E402

H, W = 1080, 1920


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, nargs="+", default=[10000, 50000])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--chol-scale", type=float, default=1.0)
    ap.add_argument("--state", default=None,
                    help="render a saved model (npz: xyz, cholesky, features) instead")
    ap.add_argument("--trained", type=int, default=0,
                    help="render the bench's frame model after this many training iterations "
                         "(trained density) instead of random splats")
    ap.add_argument("--modes", type=int, nargs="+", default=[0],
                    help="rasterizer modes (gsvc_debug_set(0)); 0 = automatic")
    ap.add_argument("--knob", type=int, nargs=2, action="append", default=[],
                    metavar=("KEY", "VALUE"), help="extra gsvc_debug_set for a second pass")
    ap.add_argument("--set", type=int, nargs=2, action="append", default=[],
                    metavar=("KEY", "VALUE"), help="gsvc_debug_set for every pass (e.g. to trace "
                    "one variant alone)")
    ap.add_argument("--stamps", action="store_true",
                    help="also run the timestamped one-wave kernel (mode 7) and print phases")
    ap.add_argument("--stamps-out", default=None,
                    help="with --stamps: save the raw per-tile stamps (us) and entry counts (npz)")
    ap.add_argument("--id-stamps", default=None, const="-", nargs="?",
                    help="stamp the production id-slab composite (knob 39) and print its phases "
                         "by entry count; optional npz path for the raw stamps")
    ap.add_argument("--proj-stamps", action="store_true",
                    help="also stamp the projection kernel's waves (knob 5) and print phases")
    args = ap.parse_args()
    args.iters = max(2, args.iters - args.iters % 2)
    lib = L.load()
    for k, v in args.set:
        if lib.gsvc_debug_set(k, v) < 0:
            raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")
    dev = torch.device("cuda:0")
    for n in args.splats:
        g = torch.Generator().manual_seed(n)
        xyz = torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5)).to(dev)
        chol = (torch.rand(n, 3, generator=g) * args.chol_scale).to(dev)
        feat = torch.rand(n, 3, generator=g).to(dev)
        bound = torch.tensor([0.5, 0.0, 0.5], device=dev)
        if args.state:
            import numpy as np
            z = np.load(args.state)
            xyz = torch.from_numpy(z["xyz"]).to(dev)
            chol = torch.from_numpy(z["cholesky"]).to(dev)
            feat = torch.from_numpy(z["features"]).to(dev)
            n = xyz.shape[0]
        if args.trained > 0:
            from gsvc_amd.frame import make_frame_model, synthetic_gt
            model = make_frame_model(H, W, n, dev, seed=1000)
            gt = synthetic_gt(H, W, 8, "cpu").to(dev)
            for it in range(1, args.trained + 1):
                model.train_iter(gt, it)
            torch.cuda.synchronize()
            xyz = model._xyz.detach().clone()
            chol = model._cholesky.detach().clone()
            feat = model.get_features.detach().clone()
            del model
        bg = torch.ones(3, device=dev)
        ws_bytes = L.size("gsvc_render_frame_workspace_bytes", n, H, W)
        ws = torch.zeros((ws_bytes,), dtype=torch.uint8, device=dev)
        meta = torch.zeros((2,), dtype=torch.int32, device=dev)
        out = torch.empty((1, 3, H, W), device=dev)
        ref = None
        counter = [0]
        passes = [(mode, None) for mode in args.modes] + [(m, kv) for kv in args.knob
                                                          for m in args.modes]
        for mode, kv in passes:
            # every pass from a zeroed workspace: the captured graph below freezes
            # each frame's parity (see the module docstring), so the counts it
            # leaves are stale, and a variant that reads the slab memory in
            # another layout (knob 24: ids) must not inherit them
            torch.cuda.synchronize()
            ws.zero_()
            lib.gsvc_debug_set(0, mode)
            if kv:
                if lib.gsvc_debug_set(kv[0], kv[1]) < 0:
                    raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")

            hint = [0]  # the density hint render.py passes: M of an earlier frame

            def frame():
                L.call("gsvc_render_frame_sum", n, L.ptr(xyz), 1, L.ptr(chol), L.ptr(bound),
                       L.ptr(feat), None, None, L.ptr(bg), H, W, counter[0], hint[0], L.ptr(meta),
                       L.ptr(ws), ws_bytes, L.ptr(out), L.stream(dev))
                counter[0] += 1

            frame()
            torch.cuda.synchronize()
            hint[0] = int(meta[0])
            # plain launches (the library call per frame): the slab entries
            # refuse graph capture (their parity slots follow the host's call
            # counter), so no graph replay here
            for _ in range(20):
                frame()
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(3):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.iters):
                    frame()
                b.record()
                torch.cuda.synchronize()
                best = min(best, a.elapsed_time(b) * 1e3 / args.iters)
            per_graph = per_launch = best
            same = True
            if ref is None:
                ref = out.clone()
            else:
                same = bool(torch.equal(out, ref))
            m = int(meta[0])
            if kv:
                lib.gsvc_debug_set(kv[0], 0)
            print(json.dumps(dict(N=n, M=m, mode=mode, knob=kv,
                                  us_per_frame=round(best, 2), fps=round(1e6 / best, 0),
                                  us_one_frame_graphs=round(per_graph, 2),
                                  us_plain_launches=round(per_launch, 2),
                                  identical=same)), flush=True)
        if args.stamps:
            import numpy as np
            ntiles = ((W + 15) // 16) * ((H + 15) // 16)
            st = torch.zeros((ntiles, 4), dtype=torch.int64, device=dev)
            lib.gsvc_debug_set_ptr(ctypes.c_void_p(st.data_ptr()))
            lib.gsvc_debug_set(0, 7)
            for _ in range(5):
                frame()
            torch.cuda.synchronize()
            lib.gsvc_debug_set(0, 0)
            lib.gsvc_debug_set_ptr(None)
            t = st.cpu().numpy().astype(np.float64) * 0.01  # 100 MHz ticks -> us
            t0 = t[:, 0].min()
            q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa
            print(json.dumps(dict(N=n, stamps="percentiles 0/10/50/90/100 (us)",
                                  start=q(t[:, 0] - t0), staged=q(t[:, 1] - t[:, 0]),
                                  blend=q(t[:, 2] - t[:, 1]), stores_drained=q(t[:, 3] - t[:, 2]),
                                  end=q(t[:, 3] - t0))), flush=True)
            if args.stamps_out:
                from gsvc_amd import ops
                from gsvc_amd.utils import bin_and_sort_for_raster
                tbs = ((W + 15) // 16, (H + 15) // 16, 1)
                with torch.no_grad():
                    means = torch.tanh(xyz)
                    L_ = chol + bound
                    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(
                        n, means, L_, H, W, tbs, 0.01)
                    _, _, bins = bin_and_sort_for_raster(n, xys, depths, radii, nth, tbs)
                counts = (bins[:, 1] - bins[:, 0]).clamp(min=0).cpu().numpy()
                np.savez_compressed(args.stamps_out, stamps_us=t - t0, counts=counts,
                                    tbx=tbs[0], tby=tbs[1])
        if args.id_stamps:
            import numpy as np
            ntiles = ((W + 15) // 16) * ((H + 15) // 16)
            st = torch.zeros((ntiles, 8), dtype=torch.int64, device=dev)
            lib.gsvc_debug_set_ptr(ctypes.c_void_p(st.data_ptr()))
            lib.gsvc_debug_set(39, 1)
            for _ in range(5):
                frame()
            torch.cuda.synchronize()
            lib.gsvc_debug_set(39, 0)
            lib.gsvc_debug_set_ptr(None)
            raw = st.cpu().numpy()
            cnt = raw[:, 5].copy()
            t = raw[:, :5].astype(np.float64) * 0.01  # 100 MHz ticks -> us
            t0 = t[:, 0].min()
            q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 99, 100)]  # noqa
            # a phase a tile skips (no entries: no ids / staging stamps) reads 0
            ok = (t[:, 1] > 0) & (t[:, 2] > 0)
            print(json.dumps(dict(N=n, id_stamps="percentiles 0/10/50/90/99/100 (us)",
                                  tiles=int(ntiles), staged_tiles=int(ok.sum()),
                                  start=q(t[:, 0] - t0),
                                  ids=q((t[ok, 1] - t[ok, 0])), records=q(t[ok, 2] - t[ok, 1]),
                                  blend=q(t[ok, 3] - t[ok, 2]), drain=q(t[:, 4] - t[:, 3]),
                                  end=q(t[:, 4] - t0))), flush=True)
            end = t[:, 4] - t0
            for lo, hi in ((0, 0), (1, 4), (5, 16), (17, 64), (65, 256), (257, 1 << 30)):
                m = (cnt >= lo) & (cnt <= hi)
                if m.any():
                    print(json.dumps(dict(count=[lo, hi], tiles=int(m.sum()),
                                          start=q(t[m, 0] - t0), end=q(end[m]))), flush=True)
            if args.id_stamps != "-":
                np.savez_compressed(args.id_stamps, stamps_us=t - t0, counts=cnt)
        if args.proj_stamps:
            import numpy as np
            waves = (n + 63) // 64
            st = torch.zeros((waves + 8, 4), dtype=torch.int64, device=dev)
            lib.gsvc_debug_set_ptr(ctypes.c_void_p(st.data_ptr()))
            lib.gsvc_debug_set(5, 1)
            for _ in range(5):
                frame()
            torch.cuda.synchronize()
            lib.gsvc_debug_set(5, 0)
            lib.gsvc_debug_set_ptr(None)
            t = st[:waves].cpu().numpy().astype(np.float64) * 0.01
            t0 = t[:, 0].min()
            q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa
            print(json.dumps(dict(N=n, proj_stamps="percentiles 0/10/50/90/100 (us)",
                                  start=q(t[:, 0] - t0), project=q(t[:, 1] - t[:, 0]),
                                  insert=q(t[:, 2] - t[:, 1]), reduce=q(t[:, 3] - t[:, 2]),
                                  end=q(t[:, 3] - t0))), flush=True)
    lib.gsvc_debug_set(0, 0)


if __name__ == "__main__":
    main()
