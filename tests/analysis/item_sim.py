"""Offline model of the band kernel's backward work layout (train.hip,
train_tile_band_kernel step 4) on a trained frame dumped by
tools/dump_trained.py: per tile and 8-row band, the entries' alpha >= 1/255
rectangles, the work items each layout makes of them, and the rounds of 64
items a wave runs -- so item layouts can be compared without a GPU.

    python tests/analysis/item_sim.py gpurun_out/trained_50k.npz

Cost model (VALU instructions per wave, calibrated against PMC
SQ_INSTS_VALU of the kernel): a round costs R + P * (its longest item's
pixels) + F per extra row of a multi-row item; a chunk costs C.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402  (checker/analysis only)

H, W = 1080, 1920


def rects(xys, conics, ids, tx0, ty0):
    """ellipse_rect (train.hip) for opacity 1: x0, x1, y0, y1 (tile-local, inclusive) or None."""
    a, b, c = conics[ids, 0], conics[ids, 1], conics[ids, 2]
    x, y = xys[ids, 0], xys[ids, 1]
    det = a * c - b * b
    lg = np.log(255.0)
    S2 = 2.0 * (lg * 1.001 + 0.01)
    with np.errstate(invalid="ignore", divide="ignore"):
        ex = np.sqrt(S2 * c / det) * 1.001 + 0.01
        ey = np.sqrt(S2 * a / det) * 1.001 + 0.01
    x0 = np.maximum(np.ceil(x - ex - tx0), 0)
    x1 = np.minimum(np.floor(x + ex - tx0), 15)
    y0 = np.maximum(np.ceil(y - ey - ty0), 0)
    y1 = np.minimum(np.floor(y + ey - ty0), 15)
    ok = (x0 <= x1) & (y0 <= y1) & (a > 0) & (det > 0)
    return x0.astype(int), x1.astype(int), y0.astype(int), y1.astype(int), ok


def layout_rows(h, w, brun=10):
    """Current layout: one item per rectangle row, two halves when w > brun."""
    items = []
    for hh, ww in zip(h, w):
        if ww > brun:
            a = (ww + 1) // 2
            items.append([(1, a), (1, ww - a)] * hh)
        else:
            items.append([(1, ww)] * hh)
    return items


def layout_multirow(h, w, target=10, brun=10):
    """Narrow rectangles: k = target // w rows per item."""
    items = []
    for hh, ww in zip(h, w):
        if ww > brun:
            a = (ww + 1) // 2
            items.append([(1, a), (1, ww - a)] * hh)
            continue
        k = max(1, target // ww)
        its = []
        left = hh
        while left > 0:
            r = min(k, left)
            its.append((r, ww))
            left -= r
        items.append(its)
    return items


def cost(items_per_entry, sort_classes, R, P, Fr, C, bounds=(9, 7, 5)):
    """VALU of one wave's chunk: items laid out entry by entry (longest class
    first when sort_classes), rounds of 64."""
    ents = list(range(len(items_per_entry)))
    if sort_classes:
        def cls(e):
            its = items_per_entry[e]
            if not its:
                return 0
            L = max(r * ww for r, ww in its)
            return sum(1 for b in bounds if L >= b)
        ents.sort(key=lambda e: -cls(e))
    flat = [it for e in ents for it in items_per_entry[e]]
    v = C
    rounds = 0
    cost.px_iter = getattr(cost, "px_iter", 0)
    cost.px_work = getattr(cost, "px_work", 0)
    for s in range(0, len(flat), 64):
        rnd = flat[s:s + 64]
        rounds += 1
        kmax = max(r for r, _ in rnd)
        px = 0
        for q in range(1, kmax + 1):
            px += max(ww for r, ww in rnd if r >= q)
        v += R + P * px + Fr * (kmax - 1)
        cost.px_iter += 64 * px
        cost.px_work += sum(r * ww for r, ww in rnd)
    return v, rounds, len(flat)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--R", type=float, default=188.0, help="VALU per round (own, seg sums, decode)")
    ap.add_argument("--P", type=float, default=30.0, help="VALU per pixel iteration")
    ap.add_argument("--F", type=float, default=14.0, help="VALU per extra row of an item")
    ap.add_argument("--C", type=float, default=0.0, help="VALU per chunk")
    ap.add_argument("--tiles", type=int, default=0, help="sample every k-th tile (0: all)")
    a = ap.parse_args()
    z = np.load(a.npz)
    tb = O.tile_bounds(H, W)
    xys, depths, radii, conics, nth = O.project_2d_forward(z["means2d"], z["L"], H, W, tb)
    m, cum = O.cumulative_intersects(nth)
    _, _, _, gids, bins = O.bin_and_sort(xys, depths, radii, cum, tb, m)
    ntiles = tb[0] * tb[1]
    step = a.tiles if a.tiles > 0 else 1
    layouts = {"rows (current)": (layout_rows, False), "rows + classes": (layout_rows, True),
               "rows brun 16 + classes 13/10/7": (lambda h, w: layout_rows(h, w, 16), (13, 10, 7)),
               "rows brun 16 + 8 classes": (lambda h, w: layout_rows(h, w, 16), (15, 13, 11, 9, 7, 5, 3)),
               "rows brun 12 + classes 11/9/7": (lambda h, w: layout_rows(h, w, 12), (11, 9, 7)),
               "multirow t10": (lambda h, w: layout_multirow(h, w, 10), False),
               "multirow t10 + classes": (lambda h, w: layout_multirow(h, w, 10), True),
               "multirow t12 + classes": (lambda h, w: layout_multirow(h, w, 12), True),
               "multirow t8 + classes": (lambda h, w: layout_multirow(h, w, 8), True),
               "rows brun 8 + classes": (lambda h, w: layout_rows(h, w, 8), True),
               "rows brun 12 + classes": (lambda h, w: layout_rows(h, w, 12), True),
               "rows brun 16 + classes": (lambda h, w: layout_rows(h, w, 16), True)}
    tot = {k: np.zeros(3) for k in layouts}
    eff = {}
    widths = []
    for t in range(0, ntiles, step):
        lo, hi = bins[t]
        ids = gids[lo:min(hi, lo + 256)]
        if len(ids) == 0:
            continue
        ty, tx = divmod(t, tb[0])
        x0, x1, y0, y1, ok = rects(xys, conics, ids, tx * 16.0, ty * 16.0)
        for band in (0, 1):
            bl, bh = 8 * band, 8 * band + 7
            r0 = np.maximum(y0, bl)
            r1 = np.minimum(y1, bh)
            hh = np.where(ok & (r0 <= r1), r1 - r0 + 1, 0)
            ww = np.where(ok, x1 - x0 + 1, 0)
            widths.extend(ww[hh > 0].tolist())
            for c0 in range(0, len(ids), 64):
                hs, ws = hh[c0:c0 + 64], ww[c0:c0 + 64]
                for k, (fn, srt) in layouts.items():
                    its = fn(hs, ws)
                    its = [x if h_ > 0 else [] for x, h_ in zip(its, hs)]
                    cost.px_iter = cost.px_work = 0
                    v, r, n = (cost(its, True, a.R, a.P, a.F, a.C, srt) if isinstance(srt, tuple)
                               else cost(its, srt, a.R, a.P, a.F, a.C))
                    tot[k] += (v, r, n)
                    eff.setdefault(k, np.zeros(2))
                    eff[k] += (cost.px_work, cost.px_iter)
    widths = np.array(widths)
    print(f"tiles sampled every {step}; entry-bands {len(widths)}; width percentiles "
          f"10/50/90: {np.percentile(widths, [10, 50, 90]).tolist()}")
    base = tot["rows (current)"][0]
    for k, (v, r, n) in tot.items():
        print(f"{k:28s} VALU {v * step / 1e6:7.2f} M  rounds {r * step / 1e3:7.1f} k  "
              f"items {n * step / 1e6:5.2f} M  lane eff {eff[k][0] / eff[k][1]:.2f}  "
              f"({100 * (v / base - 1):+.1f} %)")


if __name__ == "__main__":
    main()
