"""Offline model of the sparse composite's blend loop (raster_sum.hip,
one wave per 16x16 tile) on a trained frame: how many loop iterations a wave
runs (= the longest list among its lanes / lane groups) and how many of the
(entry, pixel) pairs it evaluates contribute, for several list granularities:

  group 4x4 rect   16 groups of 4 lanes, each lane 1x4 pixels; a group's list =
                   the entries whose alpha >= 1/255 bounding box reaches its
                   4x4 block (production, ellipse_blocks<16>)
  lane 1x4 exact   each lane its own list: the entries with alpha >= 1/255 at
                   one of its 4 pixels (exact per-pixel test)
  lane 1x4 span    each lane its own list: the entries whose alpha >= 1/255
                   ellipse crosses its 4-pixel row segment (conservative
                   row-span test, what a kernel can compute per (entry, row))
  lane 2x2 span    lanes own 2x2 quads

    python tests/analysis/lane_sim.py STATE.npz [--tiles 4]

STATE.npz: tests/analysis/train_oracle_state.py / dump_trained.py output (raw
parameters) or a fixture with state_* keys.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle as O  # noqa: E402  (analysis only)

H, W = 1080, 1920
LN255 = np.log(255.0)


def load(path):
    z = np.load(path)
    pre = "state_" if "state__xyz" in z.files else ""
    xyz = z[pre + "_xyz"]
    chol = z[pre + "_cholesky"]
    feat = z[pre + "_features_dc"]
    means = np.tanh(xyz).astype(np.float32)
    L = (chol + np.array([0.5, 0, 0.5], np.float32)).astype(np.float32)
    return means, L, feat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--tiles", type=int, default=1)
    a = ap.parse_args()
    means, L, colors = load(a.npz)
    tb = O.tile_bounds(H, W)
    xys, depths, radii, conics, nth = O.project_2d_forward(means, L, H, W, tb)
    m, cum = O.cumulative_intersects(nth)
    _, _, _, gids, bins = O.bin_and_sort(xys, depths, radii, cum, tb, m)
    ntiles = tb[0] * tb[1]
    ly, lx = np.divmod(np.arange(256), 16)
    stats = {k: [0, 0] for k in ("group 4x4 rect", "lane 1x4 exact", "lane 1x4 span",
                                 "lane 2x2 span", "pixel lists, balanced", "pixel lists, row quads")}
    valid_pairs = 0
    counts = []
    for t in range(0, ntiles, a.tiles):
        lo, hi = bins[t]
        ids = gids[lo:min(hi, lo + 256)]
        n = len(ids)
        counts.append(n)
        if n == 0:
            continue
        ty, tx = divmod(t, tb[0])
        px = (tx * 16 + lx).astype(np.float32)
        py = (ty * 16 + ly).astype(np.float32)
        cx, cy = xys[ids, 0], xys[ids, 1]
        ca, cb, cc = conics[ids, 0], conics[ids, 1], conics[ids, 2]
        dx = cx[:, None] - px[None, :]
        dy = cy[:, None] - py[None, :]
        s = 0.5 * (ca[:, None] * dx * dx + cc[:, None] * dy * dy) + cb[:, None] * dx * dy
        ok = (s >= 0) & (np.exp(-s) >= 1 / 255)  # [n, 256]
        valid_pairs += int(ok.sum())
        # production: 4x4 block rect lists (conservative bbox of the ellipse)
        det = ca * cc - cb * cb
        S2 = 2 * (LN255 * 1.001 + 0.01)
        good = (ca > 0) & (det > 0)
        ex = np.where(good, np.sqrt(S2 * cc / np.where(good, det, 1)) * 1.001 + 0.01, 1e9)
        ey = np.where(good, np.sqrt(S2 * ca / np.where(good, det, 1)) * 1.001 + 0.01, 1e9)
        u, v = cx - tx * 16, cy - ty * 16
        best = 0
        for r in range(4):
            for c in range(4):
                hit = (u + ex >= 4 * c) & (u - ex <= 4 * c + 3) & (v + ey >= 4 * r) & (v - ey <= 4 * r + 3)
                best = max(best, int(hit.sum()))
        stats["group 4x4 rect"][0] += best
        # exact per-lane lists (lane = row r, cols 4q..4q+3)
        lane_ok = ok.reshape(n, 16, 4, 4).any(axis=3).reshape(n, 64)
        stats["lane 1x4 exact"][0] += int(lane_ok.sum(axis=0).max())
        # conservative row-span per lane: for pixel row y, the ellipse's x-range
        # at that row: sigma(x) <= S  with  a/2 dx^2 + b dx dy + c/2 dy^2 <= S
        # -> dx in [(-b dy - sqrt(D)) / a, (-b dy + sqrt(D)) / a], D = b^2dy^2 - a(c dy^2 - 2S)
        S = LN255 * 1.001 + 0.01
        dyr = cy[:, None] - (ty * 16 + np.arange(16))[None, :].astype(np.float32)  # [n, 16]
        D = (cb[:, None] * dyr) ** 2 - ca[:, None] * (cc[:, None] * dyr * dyr - 2 * S)
        has = (D >= 0) & good[:, None]
        sq = np.sqrt(np.maximum(D, 0))
        # dx = cx - px  ->  px = cx - dx
        dxlo = (-cb[:, None] * dyr - sq) / np.where(good, ca, 1)[:, None]
        dxhi = (-cb[:, None] * dyr + sq) / np.where(good, ca, 1)[:, None]
        pxlo = cx[:, None] - dxhi - 0.01
        pxhi = cx[:, None] - dxlo + 0.01
        span_lane = np.zeros((n, 64), bool)
        for q in range(4):
            c0 = tx * 16 + 4 * q
            span_lane[:, q::4] = has & (pxhi >= c0) & (pxlo <= c0 + 3)
        span_lane |= ~good[:, None]
        lens = span_lane.sum(axis=0)
        stats["lane 1x4 span"][0] += int(lens.max())
        # per-pixel lists (row-span test), pixels dealt to lanes by list length
        # (snake order), each lane walking its pixels' lists one pair per
        # iteration: iterations = the longest lane total; counted in units of
        # 4 pairs per lane-iteration so the column compares with the others
        pix = np.zeros((n, 256), bool)
        for r in range(16):
            cols = tx * 16 + np.arange(16)
            pix[:, r * 16:(r + 1) * 16] = has[:, r:r + 1] & (pxhi[:, r:r + 1] >= cols[None, :]) & \
                (pxlo[:, r:r + 1] <= cols[None, :])
        pix |= ~good[:, None]
        cp = np.sort(pix.sum(axis=0))[::-1]
        lane_load = np.zeros(64, int)
        for j in range(4):
            blk = cp[64 * j:64 * (j + 1)]
            lane_load += blk if j % 2 == 0 else blk[::-1]
        stats["pixel lists, balanced"][0] += int(np.ceil(lane_load.max() / 4))
        stats["pixel lists, balanced"][1] += int(lane_load.max())
        # the same without balancing (lane = 4 consecutive pixels of a row)
        stats["pixel lists, row quads"][0] += int(np.ceil(pix.sum(axis=0).reshape(64, 4).sum(1).max() / 4))
        quad = np.zeros((n, 64), bool)
        for r2 in range(8):
            for q2 in range(8):
                rows = [2 * r2, 2 * r2 + 1]
                c0 = tx * 16 + 2 * q2
                hitq = np.zeros(n, bool)
                for rr in rows:
                    hitq |= has[:, rr] & (pxhi[:, rr] >= c0) & (pxlo[:, rr] <= c0 + 1)
                quad[:, r2 * 8 + q2] = hitq | ~good
        stats["lane 2x2 span"][0] += int(quad.sum(axis=0).max())
    counts = np.array(counts)
    print(f"tiles {len(counts)} (every {a.tiles}), entries/tile mean {counts.mean():.1f} "
          f"max {counts.max()}, M_eff {counts.sum()}")
    print(f"contributing (entry, pixel) pairs: {valid_pairs / 1e6:.2f} M")
    base = stats["group 4x4 rect"][0]
    for k, (it, _) in stats.items():
        print(f"{k:34s} wave iterations {it / 1e3:8.1f} k  pairs evaluated {it * 256 / 1e6:6.2f} M "
              f"({100 * (it / base - 1):+.1f} %)  useful {100 * valid_pairs / max(it * 256, 1):.0f} %")


if __name__ == "__main__":
    main()
