"""Training-iteration microbenchmark: GaussianVideoFrame.train_iter at
1920x1080 (BASELINE configs[2]: 50k splats by default), iterations/s.
Run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.

    python tools/tbench.py [--splats 50000] [--iters 100]
"""
from __future__ import annotations

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--op-by-op", action="store_true", help="disable the fused training step")
    ap.add_argument("--stamps", action="store_true",
                    help="also stamp the fused step's tile kernel and print phases")
    ap.add_argument("--tile-kernel", choices=["band", "wg256"], default="band",
                    help="two 8-row bands per tile (production) or the 256-thread kernel (knob 8 = 1)")
    ap.add_argument("--knob", action="append", default=[],
                    help="A/B knob K=V (gsvc_debug_set), repeatable")
    ap.add_argument("--knob-after", action="append", default=[],
                    help="knob K=V set only after the warmup (diagnostic variants that change "
                         "results must not steer the training state being measured)")
    ap.add_argument("--stamps-out", default=None,
                    help="with --stamps: save the raw per-tile stamps (us, tile order) as npz")
    ap.add_argument("--proj-stamps", action="store_true",
                    help="also stamp the projection kernel's waves (start, projected, inserted, end)")
    ap.add_argument("--splat-stamps", action="store_true",
                    help="also stamp the splat kernel's waves (start, operands, Adan, carry, M, end)")
    ap.add_argument("--rebuild-every", type=int, default=None,
                    help="steps between carried-bin rebuilds (gsvc_amd.train.CARRY_REBUILD_EVERY)")
    ap.add_argument("--order-every", type=int, default=None,
                    help="steps between splat-order sorts (gsvc_amd.train.ORDER_REFRESH_EVERY; 0: none)")
    ap.add_argument("--frozen", type=int, default=0,
                    help="after the warmup, time N gradient-only fused steps (grads_out: no "
                         "parameter update), so kernel variants are compared on one fixed state; "
                         "prints the tile kernel's event average")
    ap.add_argument("--shape", action="store_true",
                    help="also report N_vis, M, M_eff of the trained frame (op-path binning)")
    ap.add_argument("--state", default=None, metavar="NPZ:FRAME",
                    help="start from a saved model (tools/tile_counts.py --save, or a frame "
                         "exported from a video checkpoint: xyz, cholesky, features) against "
                         "frame FRAME of the textured synthetic video (dense content)")
    ap.add_argument("--pile", type=int, default=0,
                    help="move this many splats (evenly spread over the ids) onto one 5-px spot "
                         "before the warmup: a few tiles with that many candidates (the carried "
                         "lists' capacity cliff, train.hip kTrainCarryCap)")
    ap.add_argument("--channels", action="store_true",
                    help="also print HIP-event kernel averages (us) over 200 extra iterations")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    from gsvc_amd import _lib
    from gsvc_amd import train as _train
    if a.order_every is not None:
        _train.ORDER_REFRESH_EVERY = a.order_every
    if a.rebuild_every is not None:
        _train.CARRY_REBUILD_EVERY = a.rebuild_every
    _lib.load().gsvc_debug_set(8, 1 if a.tile_kernel == "wg256" else 0)
    for kv in a.knob:
        k, v = kv.split("=")
        if _lib.load().gsvc_debug_set(int(k), int(v)) < 0:
            raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    if a.state:
        import numpy as np
        from gsvc_amd.video import textured_video
        path, fr = a.state.rsplit(":", 1)
        z = np.load(path)
        a.splats = int(z["xyz"].shape[0])
        model = make_frame_model(H, W, a.splats, dev, seed=7,
                                 fused_train=False if a.op_by_op else None)
        with torch.no_grad():
            model._xyz.copy_(torch.from_numpy(z["xyz"]))
            model._cholesky.copy_(torch.from_numpy(z["cholesky"]))
            model._features_dc.copy_(torch.from_numpy(z["features"]))
        gt = textured_video(int(fr) + 1, H, W, device=dev)(int(fr))
    else:
        model = make_frame_model(H, W, a.splats, dev, seed=7,
                                 fused_train=False if a.op_by_op else None)
        gt = synthetic_gt(H, W, 8, dev)
    if a.pile:
        with torch.no_grad():
            sel = torch.linspace(0, a.splats - 1, a.pile, device=dev).long()
            g = torch.Generator(device=dev).manual_seed(3)
            model._xyz[sel] = torch.atanh(torch.full((a.pile, 2), -0.25, device=dev)
                                          + 0.005 * torch.rand(a.pile, 2, device=dev, generator=g))
            model._cholesky[sel] = torch.tensor([2.5, 0.3, 1.5], device=dev)
    for it in range(1, a.warmup + 1):
        model.train_iter(gt, it)
    torch.cuda.synchronize()
    for kv in a.knob_after:
        k, v = kv.split("=")
        if _lib.load().gsvc_debug_set(int(k), int(v)) < 0:
            raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")
    if a.frozen:
        from gsvc_amd import ops
        from gsvc_amd.train import train_step_sum
        P = model._parameters
        rgbw = model._buffers.get("rgb_W") if "rgb_W" not in P else P["rgb_W"]
        gout = torch.empty((a.splats, 9), device=dev)
        gtc = gt.reshape(-1).contiguous()

        def gstep():
            train_step_sum(P["_xyz"].data, P["_cholesky"].data, P["_features_dc"].data,
                           rgbw.data if rgbw is not None else None, False,
                           model._buffers["cholesky_bound"], model._buffers["background"], gtc,
                           H, W, grads_out=gout)
        for _ in range(10):
            gstep()
        ops.channel_timing("train_tile", True, max_launches=a.frozen, every=1, dispatch=True)
        for _ in range(a.frozen):
            gstep()
        torch.cuda.synchronize()
        ts = ops.channel_times_ms("train_tile", a.frozen)
        ops.channel_timing("train_tile", False)
        print(json.dumps(dict(frozen_steps=a.frozen, knobs=a.knob + a.knob_after,
                              train_tile_us=round(1e3 * sum(ts) / len(ts), 2))), flush=True)
        return
    t0 = time.perf_counter()
    psnr = 0.0
    blocks = []
    tb = t0
    for it in range(a.warmup + 1, a.warmup + a.iters + 1):
        _, psnr = model.train_iter(gt, it)
        if (it - a.warmup) % 100 == 0:
            tn = time.perf_counter()
            blocks.append((tn - tb) / 100)
            tb = tn
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    blocks.sort()
    block_us = dict(min=round(1e6 * blocks[0], 2), median=round(1e6 * blocks[len(blocks) // 2], 2)) \
        if blocks else {}
    shape = {}
    if a.shape:
        sys.path.insert(0, REPO)
        import bench as B
        shape = B.frame_shape(model.get_xyz.detach(), model.get_cholesky_elements.detach(),
                              model.tile_bounds)
    chan = {}
    if a.channels:
        from gsvc_amd import ops
        names = ["project", "train_tile", "train_splat"]
        for c in names:
            ops.channel_timing(c, True, max_launches=200, every=1, dispatch=True)
        for it in range(200):
            model.train_iter(gt, a.warmup + a.iters + 1 + it)
        torch.cuda.synchronize()
        for c in names:
            ts = ops.channel_times_ms(c, 200)
            chan[c] = round(1e3 * sum(ts) / max(len(ts), 1), 2)
            ops.channel_timing(c, False)
    if a.proj_stamps:
        import ctypes
        import numpy as np
        from gsvc_amd import _lib as L
        lib = L.load()
        st = torch.zeros(((a.splats + 63) // 64 + 4096, 8), dtype=torch.int64, device=dev)  # waves of any per-workgroup split
        lib.gsvc_debug_set_ptr(ctypes.c_void_p(st.data_ptr()))
        lib.gsvc_debug_set(5, 1)
        model.train_iter(gt, a.warmup + a.iters + 300)
        torch.cuda.synchronize()
        lib.gsvc_debug_set(5, 0)
        lib.gsvc_debug_set_ptr(None)
        t = st.cpu().numpy().astype(np.float64) * 0.01
        t = t[t[:, 3] > 0]
        t0 = t[:, 0].min()
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa
        print(json.dumps(dict(proj_stamps="percentiles 0/10/50/90/100 (us)", waves=int(len(t)),
                              start=q(t[:, 0] - t0), project=q(t[:, 1] - t[:, 0]),
                              insert=q(t[:, 2] - t[:, 1]), reduce=q(t[:, 3] - t[:, 2]),
                              window=q(t[:, 4] - t[:, 1]),
                              lds_count=q((t[:, 5] - t[:, 4])[t[:, 6] > 0]),
                              base_atomics=q((t[:, 6] - t[:, 5])[t[:, 6] > 0]),
                              slab_stores=q((t[:, 7] - t[:, 6])[t[:, 6] > 0]),
                              windowed_waves=int((t[:, 6] > 0).sum()),
                              end=q(t[:, 3] - t0))), flush=True)
    if a.splat_stamps:
        import ctypes
        import numpy as np
        from gsvc_amd import _lib as L
        lib = L.load()
        st = torch.zeros(((a.splats + 255) // 256 * 4 + 8, 8), dtype=torch.int64, device=dev)
        lib.gsvc_debug_set_ptr(ctypes.c_void_p(st.data_ptr()))
        lib.gsvc_debug_set(5, 4)
        model.train_iter(gt, a.warmup + a.iters + 400)
        torch.cuda.synchronize()
        lib.gsvc_debug_set(5, 0)
        lib.gsvc_debug_set_ptr(None)
        t = st.cpu().numpy().astype(np.float64) * 0.01
        loss_wg = t[:4]
        t = t[4:]
        t = t[t[:, 5] > 0]
        t0 = min(t[:, 0].min(), loss_wg[loss_wg[:, 0] > 0][:, 0].min())
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa
        print(json.dumps(dict(splat_stamps="percentiles 0/10/50/90/100 (us)", waves=int(len(t)),
                              start=q(t[:, 0] - t0), operands=q(t[:, 1] - t[:, 0]),
                              adan=q(t[:, 2] - t[:, 1]), carry=q(t[:, 3] - t[:, 2]),
                              m_add=q(t[:, 4] - t[:, 3]), drain=q(t[:, 5] - t[:, 4]),
                              end=q(t[:, 5] - t0),
                              loss_wg_end=round(float(loss_wg[:, 5].max() - t0), 2))), flush=True)
    if a.stamps:
        import ctypes
        import numpy as np
        from gsvc_amd import _lib as L
        lib = L.load()
        ntiles = ((W + 15) // 16) * ((H + 15) // 16)
        st = torch.zeros((ntiles, 8), dtype=torch.int64, device=dev)
        lib.gsvc_debug_set_ptr(ctypes.c_void_p(st.data_ptr()))
        lib.gsvc_debug_set(5, 2 if a.tile_kernel == "wg256" else 3)
        model.train_iter(gt, a.warmup + a.iters + 1)
        torch.cuda.synchronize()
        lib.gsvc_debug_set(5, 0)
        lib.gsvc_debug_set_ptr(None)
        t = st.cpu().numpy().astype(np.float64) * 0.01
        if a.stamps_out:
            raw = st.cpu().numpy()
            np.savez_compressed(a.stamps_out, stamps_us=raw[:, :6] * 0.01 - t[t[:, 5] > 0][:, 0].min(),
                                counts=raw[:, 6], tbx=(W + 15) // 16, tby=(H + 15) // 16)
        t = t[t[:, 5] > 0]
        t0 = t[:, 0].min()
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa
        names = (("staged", "forward", "scan", "items", "atomics") if a.tile_kernel == "wg256" else
                 ("ordered", "forward", "loss", "backward", "end"))
        rec = dict(stamps="percentiles 0/10/50/90/100 (us)", kernel=a.tile_kernel,
                   tiles=int(len(t)), start=q(t[:, 0] - t0))
        for k, nm in enumerate(names):
            rec[nm] = q(t[:, k + 1] - t[:, k])
        rec.update(life=q(t[:, 5] - t[:, 0]), end=q(t[:, 5] - t0))
        print(json.dumps(rec), flush=True)
        # the same phases for the tiles of the first wave of workgroups (started
        # within 5 us) and for the rest
        early = (t[:, 0] - t0) < 5.0
        for lab, sel in (("first_round", early), ("later", ~early)):
            if sel.sum():
                ts = t[sel]
                print(json.dumps({lab: dict(tiles=int(sel.sum()), **{
                    nm: q(ts[:, k + 1] - ts[:, k]) for k, nm in enumerate(names)},
                    t_start=q(ts[:, 0] - t0), t_end=q(ts[:, 5] - t0))}), flush=True)
        if a.tile_kernel == "band":
            # medians per entry-count bucket (stamp slot 6 = the tile's count)
            cnt = st.cpu().numpy()[:, 6][st.cpu().numpy()[:, 5] > 0]
            by = {}
            for lo, hi in ((0, 16), (17, 32), (33, 64), (65, 128), (129, 256), (257, 1 << 30)):
                sel = (cnt >= lo) & (cnt <= hi)
                if sel.sum() == 0:
                    continue
                ts = t[sel]
                by[f"{lo}-{hi}"] = dict(tiles=int(sel.sum()), **{
                    nm: round(float(np.median(ts[:, k + 1] - ts[:, k])), 2)
                    for k, nm in enumerate(names)}, life=round(float(np.median(ts[:, 5] - ts[:, 0])), 2))
            print(json.dumps(dict(by_count=by, count_mean=round(float(cnt.mean()), 2))), flush=True)
    print(json.dumps(dict(splats=a.splats, tile_kernel=a.tile_kernel,
                          fused_train=model.fused_steps > 0, iters_per_s=round(1 / dt, 1),
                          ms_per_iter=round(1e3 * dt, 4), psnr=round(psnr, 3),
                          us_per_iter_100=block_us, knobs=a.knob,
                          order_every=_train.ORDER_REFRESH_EVERY, shape=shape,
                          kernel_us=chan)), flush=True)


if __name__ == "__main__":
    main()
