"""Offline model of the band kernel's forward (train.hip step 2, and the
render's banded composite) on a trained frame dumped by tools/dump_trained.py:
per tile and 8-row band, how many entry iterations a wave runs when its lanes
are split into groups that each walk only the entries whose alpha >= 1/255
rectangle reaches the group's sub-rectangle (iterations = the longest group
list), against the whole band walking the band's union (the current kernel).

    python tests/analysis/fwd_sim.py gpurun_out/trained_50k.npz [--tiles 4]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from oracle import oracle as O  # noqa: E402  (analysis only)
from item_sim import rects, H, W  # noqa: E402

# group sub-rectangles of one 8-row x 16-col band: (row0, row1, col0, col1) inclusive
SHAPES = {
    "band 8x16 (current)": [(0, 7, 0, 15)],
    "2 groups 8x8": [(0, 7, 0, 7), (0, 7, 8, 15)],
    "2 groups 4x16": [(0, 3, 0, 15), (4, 7, 0, 15)],
    "4 groups 4x8": [(r, r + 3, c, c + 7) for r in (0, 4) for c in (0, 8)],
    "4 groups 2x16": [(r, r + 1, 0, 15) for r in (0, 2, 4, 6)],
    "4 groups 8x4": [(0, 7, c, c + 3) for c in (0, 4, 8, 12)],
    "8 groups 4x4": [(r, r + 3, c, c + 3) for r in (0, 4) for c in (0, 4, 8, 12)],
    "8 groups 2x8": [(r, r + 1, c, c + 7) for r in (0, 2, 4, 6) for c in (0, 8)],
}
# one wave over the whole 16x16 tile (the sparse composite, 4 pixels per lane)
TILE_SHAPES = {
    "tile 16x16 (sparse, current)": [(0, 15, 0, 15)],
    "tile: 16 groups 4x4": [(r, r + 3, c, c + 3) for r in (0, 4, 8, 12) for c in (0, 4, 8, 12)],
    "tile: 8 groups 4x8": [(r, r + 3, c, c + 7) for r in (0, 4, 8, 12) for c in (0, 8)],
    "tile: 8 groups 8x4": [(r, r + 7, c, c + 3) for r in (0, 8) for c in (0, 4, 8, 12)],
    "tile: 4 groups 8x8": [(r, r + 7, c, c + 7) for r in (0, 8) for c in (0, 8)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--tiles", type=int, default=0, help="sample every k-th tile (0: all)")
    a = ap.parse_args()
    z = np.load(a.npz)
    tb = O.tile_bounds(H, W)
    xys, depths, radii, conics, nth = O.project_2d_forward(z["means2d"], z["L"], H, W, tb)
    m, cum = O.cumulative_intersects(nth)
    _, _, _, gids, bins = O.bin_and_sort(xys, depths, radii, cum, tb, m)
    ntiles = tb[0] * tb[1]
    step = a.tiles if a.tiles > 0 else 1
    iters = {k: 0 for k in SHAPES}
    titers = {k: 0 for k in TILE_SHAPES}
    inside = 0
    for t in range(0, ntiles, step):
        lo, hi = bins[t]
        ids = gids[lo:min(hi, lo + 256)]
        if len(ids) == 0:
            continue
        ty, tx = divmod(t, tb[0])
        x0, x1, y0, y1, ok = rects(xys, conics, ids, tx * 16.0, ty * 16.0)
        for k, groups in TILE_SHAPES.items():
            best = 0
            for (r0, r1, c0, c1) in groups:
                hit = ok & (y0 <= r1) & (y1 >= r0) & (x0 <= c1) & (x1 >= c0)
                best = max(best, int(hit.sum()))
            titers[k] += best
        for band in (0, 1):
            b0 = 8 * band
            for k, groups in SHAPES.items():
                best = 0
                for (r0, r1, c0, c1) in groups:
                    hit = ok & (y0 <= b0 + r1) & (y1 >= b0 + r0) & (x0 <= c1) & (x1 >= c0)
                    best = max(best, int(hit.sum()))
                iters[k] += best
            r0 = np.maximum(y0, b0)
            r1 = np.minimum(y1, b0 + 7)
            inside += int(np.sum(np.where(ok & (r0 <= r1), (r1 - r0 + 1) * (x1 - x0 + 1), 0)))
    base = iters["band 8x16 (current)"]
    print(f"tiles every {step}: (entry, pixel) pairs inside rectangles {inside * step / 1e6:.2f} M")
    for k, v in iters.items():
        print(f"{k:22s} wave iterations {v * step / 1e3:8.1f} k  pairs evaluated "
              f"{v * step * 128 / 1e6:6.2f} M  ({100 * (v / base - 1):+.1f} %)")
    tb0 = titers["tile 16x16 (sparse, current)"]
    for k, v in titers.items():
        print(f"{k:28s} wave iterations {v * step / 1e3:8.1f} k  pairs evaluated "
              f"{v * step * 256 / 1e6:6.2f} M  ({100 * (v / tb0 - 1):+.1f} %)")


if __name__ == "__main__":
    main()
