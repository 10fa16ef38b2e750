"""How fast do the training step's tile bins change at trained density?

Trains the bench's 1080p / 50k frame (seed 1000, --settle iterations), then
for --steps more fused steps records every splat's tile bbox (common.h
tile_bbox of the projection's xys / radii) after each step, and reports per
step: splats whose bbox changed, (splat, tile) pairs added to / dropped from
the bins, and -- for a bin that only ever grows between full rebuilds -- the
stale pairs it carries K steps after a rebuild (candidates / true pairs).

  python tools/bin_drift.py [--settle 2000] [--steps 128]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def bboxes(model):
    from gsvc_amd.project_gaussians_2d import project_gaussians_2d
    with torch.no_grad():
        xys, _, radii, _, _ = project_gaussians_2d(model.get_xyz, model.get_cholesky_elements,
                                                   model.H, model.W, model.tile_bounds)
    tbx, tby = model.tile_bounds[0], model.tile_bounds[1]
    t = xys / 16.0
    r = radii.float() / 16.0
    x0 = (t[:, 0] - r).trunc().clamp(0, tbx).int()
    x1 = ((t[:, 0] + r) + 1.0).trunc().clamp(0, tbx).int()
    y0 = (t[:, 1] - r).trunc().clamp(0, tby).int()
    y1 = ((t[:, 1] + r) + 1.0).trunc().clamp(0, tby).int()
    vis = radii > 0
    b = torch.stack([x0, y0, x1, y1], 1)
    b[~vis] = 0
    return b


def area(b):
    return ((b[:, 2] - b[:, 0]).clamp(min=0) * (b[:, 3] - b[:, 1]).clamp(min=0)).long()


def inter(a, b):
    lo = torch.maximum(a[:, :2], b[:, :2])
    hi = torch.minimum(a[:, 2:], b[:, 2:])
    return ((hi[:, 0] - lo[:, 0]).clamp(min=0) * (hi[:, 1] - lo[:, 1]).clamp(min=0)).long()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settle", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--splats", type=int, default=50000)
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    model = make_frame_model(1080, 1920, a.splats, dev, seed=1000)
    gt = synthetic_gt(1080, 1920, 8, "cpu").to(dev)
    it = 0
    for _ in range(a.settle):
        it += 1
        model.train_iter(gt, it)
    b0 = bboxes(model)
    prev = b0
    # the union bin since the rebuild, as a per-splat bbox hull (an upper bound
    # of a grow-only bin's pairs: the hull of every bbox held so far)
    hull = b0.clone()
    rows = []
    for k in range(1, a.steps + 1):
        it += 1
        model.train_iter(gt, it)
        b = bboxes(model)
        changed = (b != prev).any(1)
        added = int((area(b) - inter(b, prev)).sum())
        dropped = int((area(prev) - inter(b, prev)).sum())
        hull[:, :2] = torch.minimum(hull[:, :2], b[:, :2])
        hull[:, 2:] = torch.maximum(hull[:, 2:], b[:, 2:])
        true_pairs = int(area(b).sum())
        rows.append({"step": k, "splats_changed": int(changed.sum()), "pairs_added": added,
                     "pairs_dropped": dropped, "pairs": true_pairs,
                     "hull_pairs": int(area(hull).sum()),
                     "max_shift_px": float((b - prev).abs().max()) * 16})
        prev = b
    for r in rows:
        if r["step"] in (1, 2, 4, 8, 16, 32, 64, 96, 128) or r["step"] == a.steps:
            print(json.dumps(r), flush=True)
    tot = {"mean_splats_changed": sum(r["splats_changed"] for r in rows) / len(rows),
           "mean_pairs_added": sum(r["pairs_added"] for r in rows) / len(rows)}
    print(json.dumps(tot))


if __name__ == "__main__":
    main()
