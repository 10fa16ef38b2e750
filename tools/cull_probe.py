"""Debug: pixels where the banded composite (knob 0 = 2) and the sparse one
disagree on a video-driver checkpoint's frame; per such pixel, the tile's
entries (first 256 by id) whose alpha at the pixel passes the reference test
(sigma >= 0, min(1, exp(-sigma)) >= 1/255) together with the culling
rectangles the kernels use (cull.h ellipse_blocks: the 4x4 block of the
pixel, in float32 as written, IEEE and approximate) -- a passing entry whose
block is culled is a culling error.

    python tools/cull_probe.py CHECKPOINT.pth frame_116
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

f32 = np.float32


def blocks_hit(x, y, a, b, c, bx0, by0, px, py):
    """ellipse_blocks' test for the 4x4 block holding pixel (px, py), float32."""
    det = f32(f32(a * c) - f32(b * b))
    if not (a > 0 and det > 0):
        return True, None, None, float(det)
    lg = f32(np.log(f32(255.0)))
    S2 = f32(2.0) * f32(f32(lg * f32(1.001)) + f32(0.01))
    ex = f32(f32(np.sqrt(f32(f32(S2 * c) / det))) * f32(1.001)) + f32(0.01)
    ey = f32(f32(np.sqrt(f32(f32(S2 * a) / det))) * f32(1.001)) + f32(0.01)
    u, v = f32(x - bx0), f32(y - by0)
    k, r = int((px - bx0) // 4), int((py - by0) // 4)
    hit = (u + ex >= 4 * k) and (u - ex <= 4 * k + 3) and (v + ey >= 4 * r) and (v - ey <= 4 * r + 3)
    return bool(hit), float(ex), float(ey), float(det)


def main():
    from conftest import knobs
    from gsvc_amd import ops
    from gsvc_amd.render import render_frame_sum
    dev = torch.device("cuda:0")
    sd = torch.load(sys.argv[1], weights_only=True, map_location="cpu")[sys.argv[2]]
    H, W = 1080, 1920
    xyz, chol, feat = (sd[k].to(dev) for k in ("_xyz", "_cholesky", "_features_dc"))
    n = xyz.shape[0]
    bound = torch.tensor([0.5, 0.0, 0.5], device=dev)
    bg = torch.ones(3, device=dev)
    with torch.no_grad():
        sparse = render_frame_sum(xyz, chol, feat, H, W, bg, cholesky_bound=bound)
        with knobs((0, 2)):
            banded = render_frame_sum(xyz, chol, feat, H, W, bg, cholesky_bound=bound)
        tb = ((W + 15) // 16, (H + 15) // 16, 1)
        xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(
            n, torch.tanh(xyz), chol + bound, H, W, tb, 0.01)
    bad = (sparse != banded).any(1)[0]
    ys, xs = torch.nonzero(bad, as_tuple=True)
    X, R, C = xys.cpu().numpy(), radii.cpu().numpy(), conics.cpu().numpy()
    col = feat.cpu().numpy()
    for py, px in zip(ys.tolist(), xs.tolist()):
        tx, ty = px // 16, py // 16
        # the tile's entries: splats whose tile bbox covers it, ascending id
        tcx, tcy, tr = X[:, 0] / 16, X[:, 1] / 16, R / 16
        x0 = np.clip(np.trunc(tcx - tr), 0, tb[0]); x1 = np.clip(np.trunc(tcx + tr + 1), 0, tb[0])
        y0 = np.clip(np.trunc(tcy - tr), 0, tb[1]); y1 = np.clip(np.trunc(tcy + tr + 1), 0, tb[1])
        ids = np.nonzero((R > 0) & (x0 <= tx) & (tx < x1) & (y0 <= ty) & (ty < y1))[0][:256]
        rows = []
        for g in ids:
            x, y = f32(X[g, 0]), f32(X[g, 1])
            a, b, c = (f32(v) for v in C[g])
            dx, dy = f32(x - f32(px)), f32(y - f32(py))
            sigma = f32(f32(0.5) * f32(f32(a * dx * dx) + f32(c * dy * dy))) + f32(b * dx * dy)
            alpha = min(1.0, float(np.exp(-np.float64(sigma))))
            ok = sigma >= 0 and alpha >= 1 / 255
            t16 = blocks_hit(x, y, a, b, c, f32(tx * 16), f32(ty * 16), px, py)
            t8 = blocks_hit(x, y, a, b, c, f32(tx * 16), f32(ty * 16 + (8 if py % 16 >= 8 else 0)),
                            px, py)
            if ok and not (t16[0] and t8[0]):
                rows.append(dict(id=int(g), sigma=float(sigma), alpha=alpha, blk16=t16[0],
                                 blk8=t8[0], ex=t16[1], ey=t16[2], det=t16[3],
                                 conic=[float(a), float(b), float(c)], xy=[float(x), float(y)],
                                 rgb=col[g].tolist()))
        print(json.dumps(dict(pixel=[px, py], tile=[tx, ty], entries=len(ids),
                              sparse=sparse[0, :, py, px].tolist(), banded=banded[0, :, py, px].tolist(),
                              culled_contributors=rows)), flush=True)


if __name__ == "__main__":
    main()
