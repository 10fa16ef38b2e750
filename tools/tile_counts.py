"""Tile occupancy of trained P-frame models on the textured synthetic video
(gsvc_amd.video.textured_video): a chain of --frames FrameTrainer runs at
1920x1080 (fixed --iterations per frame, early stop off, as video600's
configs 4/5 stand-in), printing per frame the training time and the
distribution of per-tile intersection counts (the reference's tile bbox of
each splat, project_gaussians_2d's xys / radii) -- how many tiles carry more
than the 256 entries the sum rasterizer blends (config.h BLOCK_SIZE), the
case the kernels resolve from more than one slab's worth of candidates.

    python tools/tile_counts.py [--frames 40] [--iterations 2000] [--splats 50000]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def tile_counts(xys, radii, H, W):
    """Per-tile count of splats whose tile bbox covers the tile (common.h
    tile_bbox: [trunc(c / 16 - r / 16), trunc(c / 16 + r / 16 + 1)) clamped)."""
    tbx, tby = (W + 15) // 16, (H + 15) // 16
    vis = radii > 0
    c, r = xys[vis].float(), radii[vis].float()
    tc, tr = c / 16, r / 16
    x0 = (tc[:, 0] - tr).trunc().clamp(0, tbx).long()
    x1 = (tc[:, 0] + tr + 1).trunc().clamp(0, tbx).long()
    y0 = (tc[:, 1] - tr).trunc().clamp(0, tby).long()
    y1 = (tc[:, 1] + tr + 1).trunc().clamp(0, tby).long()
    # 2D difference array over the tile grid, then prefix sums
    d = torch.zeros((tby + 1, tbx + 1), dtype=torch.int64, device=xys.device)
    ok = (x1 > x0) & (y1 > y0)
    x0, x1, y0, y1 = x0[ok], x1[ok], y0[ok], y1[ok]
    flat = d.view(-1)
    s = tbx + 1
    flat.index_add_(0, y0 * s + x0, torch.ones_like(x0))
    flat.index_add_(0, y0 * s + x1, -torch.ones_like(x0))
    flat.index_add_(0, y1 * s + x0, -torch.ones_like(x0))
    flat.index_add_(0, y1 * s + x1, torch.ones_like(x0))
    return d.cumsum(0).cumsum(1)[:tby, :tbx].reshape(-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--iterations", type=int, default=2000)
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--save", default=None, help="npz of the last frame's model (xyz, cholesky, features)")
    a = ap.parse_args()
    from gsvc_amd import ops
    from gsvc_amd.video import FrameTrainer, textured_video
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    frame = textured_video(a.frames, H, W, device=dev)
    gmodel = None
    for f in range(a.frames):
        img = frame(f)
        tr = FrameTrainer(img, f, "L2", a.splats, a.splats, a.iterations, 1e-3, 100,
                          trained_model=gmodel, isdensity=False, isremoval=False,
                          early_stop=False)
        t0 = time.time()
        r = tr.train()
        wall = time.time() - t0
        gmodel = r.pop("model")
        m = tr.model
        with torch.no_grad():
            xys, _, radii, _, _ = ops.project_gaussians_2d_forward(
                m._xyz.shape[0], m.get_xyz, m.get_cholesky_elements, H, W,
                ((W + 15) // 16, (H + 15) // 16, 1), 0.01)
            cnt = tile_counts(xys, radii, H, W)
        c = cnt.cpu()
        print(json.dumps(dict(frame=f, psnr=round(r["psnr"], 3), train_s=round(r["training_time"], 3),
                              wall_s=round(wall, 3), M=int(c.sum()), max=int(c.max()),
                              over256=int((c > 256).sum()), over512=int((c > 512).sum()),
                              over1024=int((c > 1024).sum()), over2048=int((c > 2048).sum()),
                              p99=int(c.float().quantile(0.99)))), flush=True)
    if a.save:
        import numpy as np
        np.savez_compressed(a.save, xyz=m._xyz.detach().cpu().numpy(),
                            cholesky=m._cholesky.detach().cpu().numpy(),
                            features=m._features_dc.detach().cpu().numpy())


if __name__ == "__main__":
    main()
