"""Offline estimate for the training tile kernel's backward (train.hip step 4)
at the bench's trained state (tests/golden/train_state_1080p_n50k.npz): how
many pixel-loop iterations the per-row work items take when an item walks its
entry's whole alpha >= 1/255 rectangle row (today) versus only the row's exact
span of sigma <= the cut (the quadratic's roots, with a margin).  A round of 64
items costs its longest item; items are laid out longest first in four classes
as the kernel does.  Analysis only (CPU).

    python tests/analysis/span_sim.py [--tiles 8160]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

H, W = 1080, 1920
CUT = np.float32(5.5412636)  # common.h kSigmaCutBits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=8160)
    a = ap.parse_args()
    z = np.load(os.path.join(REPO, "tests", "golden", "train_state_1080p_n50k.npz"))
    means = np.tanh(z["state__xyz"]).astype(np.float32)
    L = (z["state__cholesky"] + np.array([0.5, 0.0, 0.5], np.float32)).astype(np.float32)
    tb = O.tile_bounds(H, W)
    xys, depths, radii, conics, nth = O.project_2d_forward(means, L, H, W, tb)
    m, cum = O.cumulative_intersects(nth)
    _, _, _, gids, bins = O.bin_and_sort(xys, depths, radii, cum, tb, m)
    tbx = tb[0]
    tot = {"rect": 0, "span": 0, "span_cls": 0}
    pix = {"rect": 0, "span": 0}
    for tile in range(min(a.tiles, len(bins))):
        b0, b1 = bins[tile]
        ids = gids[b0:min(b1, b0 + 256)]
        if len(ids) == 0:
            continue
        ty, tx = divmod(tile, tbx)
        tx0, ty0 = tx * 16.0, ty * 16.0
        x, y = xys[ids, 0].astype(np.float64), xys[ids, 1].astype(np.float64)
        ca, cb, cc = (conics[ids, k].astype(np.float64) for k in range(3))
        det = ca * cc - cb * cb
        S2 = 2.0 * (np.log(255.0) * 1.001 + 0.01)
        with np.errstate(invalid="ignore", divide="ignore"):
            ex = np.sqrt(S2 * cc / det) * 1.001 + 0.01
            ey = np.sqrt(S2 * ca / det) * 1.001 + 0.01
        rx0 = np.maximum(np.ceil(x - ex - tx0), 0)
        rx1 = np.minimum(np.floor(x + ex - tx0), 15)
        ry0 = np.maximum(np.ceil(y - ey - ty0), 0)
        ry1 = np.minimum(np.floor(y + ey - ty0), 15)
        ok = (rx0 <= rx1) & (ry0 <= ry1) & (ca > 0) & (det > 0)
        for band in range(2):
            ylo, yhi = 8 * band, 8 * band + 7
            items_r, items_s, cls = [], [], []
            for e in np.nonzero(ok)[0]:
                r0, r1 = max(ry0[e], ylo), min(ry1[e], yhi)
                if r0 > r1:
                    continue
                w = int(rx1[e] - rx0[e] + 1)
                c = 3 if w >= 9 else (2 if w >= 7 else (1 if w >= 5 else 0))
                ent_r, ent_s = [], []
                for row in range(int(r0), int(r1) + 1):
                    dy = y[e] - (ty0 + row)
                    ha, hc = 0.5 * ca[e], 0.5 * cc[e]
                    # sigma(dx) = ha dx^2 + b dy dx + hc dy^2 <= CUT
                    A, B, C = ha, cb[e] * dy, hc * dy * dy - CUT
                    D = B * B - 4 * A * C
                    if D < 0:
                        s = 0
                    else:
                        sq = np.sqrt(D)
                        lo, hi = (-B - sq) / (2 * A), (-B + sq) / (2 * A)
                        # pixels px with x - px in [lo, hi]: px in [x - hi, x - lo], margins
                        pl = np.ceil(x[e] - hi - tx0 - 0.01 - 1e-3 * abs(hi))
                        pr = np.floor(x[e] - lo - tx0 + 0.01 + 1e-3 * abs(lo))
                        pl, pr = max(pl, rx0[e]), min(pr, rx1[e])
                        s = int(max(0, pr - pl + 1))
                    ent_r.append(w)
                    ent_s.append(s)
                items_r.append(ent_r)
                items_s.append(ent_s)
                cls.append(c)
            order = np.argsort(-np.array(cls), kind="stable")
            flat_r = [l for i in order for l in items_r[i]]
            flat_s = [l for i in order for l in items_s[i]]
            pix["rect"] += sum(flat_r)
            pix["span"] += sum(flat_s)
            for k in range(0, len(flat_r), 64):
                tot["rect"] += max(flat_r[k:k + 64])
                tot["span"] += max(flat_s[k:k + 64])
            # span classes by the entry's longest span
            cls2 = [max(s) if s else 0 for s in items_s]
            order2 = np.argsort(-np.array(cls2), kind="stable")
            flat2 = [l for i in order2 for l in items_s[i]]
            for k in range(0, len(flat2), 64):
                tot["span_cls"] += max(flat2[k:k + 64])
    print("pixels in items: rect", pix["rect"], "span", pix["span"],
          f"({pix['span'] / pix['rect']:.3f})")
    print("sum over rounds of the longest item: rect", tot["rect"], "span", tot["span"],
          f"({tot['span'] / tot['rect']:.3f})", "span classes", tot["span_cls"],
          f"({tot['span_cls'] / tot['rect']:.3f})")


if __name__ == "__main__":
    main()
