"""Offline estimate (CPU, the C oracle's projection of the bench's trained
1080p / 50k state, tests/golden/train_state_1080p_n50k.npz): blend-loop trips
of the tile kernels' forward with the lane-group lists (a list per 4x4 pixel
block, the wave looping to the longest) against per-lane lists (each lane its
own entries, the wave looping to the lane with the most).  Prints the trip
counts summed over the frame for the training kernel's bands (2 px per lane)
and the render's one-wave tiles (4 px per lane).  Analysis only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

H, W = 1080, 1920
z = np.load(os.path.join(REPO, "tests/golden/train_state_1080p_n50k.npz"))
means = np.tanh(z["state__xyz"]).astype(np.float32)
L = (z["state__cholesky"] + np.array([0.5, 0, 0.5], np.float32)).astype(np.float32)
O.lib()
tb = O.tile_bounds(H, W)
xys, depths, radii, conics, nth = O.project_2d_forward(means, L, H, W, tb)
tbx, tby = tb[0], tb[1]
n = len(xys)
lg = np.log(255.0)
S2 = 2.0 * (lg * 1.001 + 0.01)
a, b, c = conics[:, 0], conics[:, 1], conics[:, 2]
det = a * c - b * b
ex = np.sqrt(np.maximum(S2 * c / det, 0)) * 1.001 + 0.01
ey = np.sqrt(np.maximum(S2 * a / det, 0)) * 1.001 + 0.01
tcx, tcy, tr = xys[:, 0] / 16, xys[:, 1] / 16, radii / 16
x0t = np.clip((tcx - tr).astype(np.int64), 0, tbx); x1t = np.clip((tcx + tr + 1).astype(np.int64), 0, tbx)
y0t = np.clip((tcy - tr).astype(np.int64), 0, tby); y1t = np.clip((tcy + tr + 1).astype(np.int64), 0, tby)
tiles = [[] for _ in range(tbx * tby)]
for i in np.nonzero(radii > 0)[0]:
    for ty in range(y0t[i], y1t[i]):
        for tx in range(x0t[i], x1t[i]):
            tiles[ty * tbx + tx].append(i)
tr_cur = tr_new = rd_cur = rd_new = 0
for t, ids in enumerate(tiles):
    ids = sorted(ids)[:256]
    if not ids:
        continue
    ty, tx = divmod(t, tbx)
    ids = np.array(ids)
    X0 = np.maximum(np.ceil(xys[ids, 0] - ex[ids] - 16 * tx), 0)
    X1 = np.minimum(np.floor(xys[ids, 0] + ex[ids] - 16 * tx), 15)
    Y0 = np.maximum(np.ceil(xys[ids, 1] - ey[ids] - 16 * ty), 0)
    Y1 = np.minimum(np.floor(xys[ids, 1] + ey[ids] - 16 * ty), 15)
    ok = (X0 <= X1) & (Y0 <= Y1)
    X0, X1, Y0, Y1 = X0[ok], X1[ok], Y0[ok], Y1[ok]
    for c0 in range(0, len(X0), 64):
        sl = slice(c0, c0 + 64)
        x0, x1, y0, y1 = X0[sl], X1[sl], Y0[sl], Y1[sl]
        # per pixel: entries covering it
        rows = np.arange(16)[:, None, None]
        cols = np.arange(16)[None, :, None]
        cov = (y0 <= rows) & (y1 >= rows) & (x0 <= cols) & (x1 >= cols)  # [16,16,E]
        # training bands: 8 rows, lanes = (row, col pair); groups = 4x4 blocks
        for band in range(2):
            r = slice(8 * band, 8 * band + 8)
            pair = cov[r].reshape(8, 8, 2, -1).any(axis=2)  # [8 rows, 8 pairs, E]
            tr_new += pair.sum(axis=2).max()
            blk = cov[r].reshape(2, 4, 4, 4, -1).any(axis=(1, 3))  # [2,4,E]
            tr_cur += blk.sum(axis=2).max()
        # render: one wave, lanes = (row, 4-px quad); groups = 4x4 blocks
        quad = cov.reshape(16, 4, 4, -1).any(axis=2)
        rd_new += quad.sum(axis=2).max()
        blk = cov.reshape(4, 4, 4, 4, -1).any(axis=(1, 3))
        rd_cur += blk.sum(axis=2).max()
print(dict(train_band_trips_groups=int(tr_cur), train_band_trips_lanes=int(tr_new),
           render_trips_groups=int(rd_cur), render_trips_lanes=int(rd_new)))

# backward: work items = an entry's rectangle rows inside the band, laid out
# longest class first (9+, 7-8, 5-6, <= 4), rounds of 64 items; a round's pixel
# loop runs as long as its longest item
def classes(ln):
    return np.where(ln >= 9, 3, np.where(ln >= 7, 2, np.where(ln >= 5, 1, 0)))


used = paid = paid_exact = rounds_sep = rounds_pool = 0
for t, ids in enumerate(tiles):
    ids = sorted(ids)[:256]
    if not ids:
        continue
    ty, tx = divmod(t, tbx)
    ids = np.array(ids)
    X0 = np.maximum(np.ceil(xys[ids, 0] - ex[ids] - 16 * tx), 0)
    X1 = np.minimum(np.floor(xys[ids, 0] + ex[ids] - 16 * tx), 15)
    Y0 = np.maximum(np.ceil(xys[ids, 1] - ey[ids] - 16 * ty), 0)
    Y1 = np.minimum(np.floor(xys[ids, 1] + ey[ids] - 16 * ty), 15)
    ok = (X0 <= X1) & (Y0 <= Y1)
    X0, X1, Y0, Y1 = X0[ok], X1[ok], Y0[ok], Y1[ok]
    for c0 in range(0, len(X0), 64):
        nitems = [0, 0]
        for band in range(2):
            lo, hi = 8 * band, 8 * band + 7
            items = []
            for e in range(c0, min(c0 + 64, len(X0))):
                r0, r1 = max(Y0[e], lo), min(Y1[e], hi)
                if r0 <= r1:
                    items.append((int(r1 - r0 + 1), int(X1[e] - X0[e] + 1)))
            if not items:
                continue
            nr = np.array([k for k, _ in items]); ln = np.array([w for _, w in items])
            nitems[band] = int(nr.sum())
            cl = classes(ln)
            order = np.argsort(-cl, kind="stable")
            seq = np.repeat(ln[order], nr[order])
            used += seq.sum()
            for b0 in range(0, len(seq), 64):
                paid += 64 * seq[b0:b0 + 64].max()
            seq2 = np.sort(np.repeat(ln, nr))[::-1]
            for b0 in range(0, len(seq2), 64):
                paid_exact += 64 * seq2[b0:b0 + 64].max()
        rounds_sep += sum((k + 63) // 64 for k in nitems)
        rounds_pool += 2 * ((sum(nitems) + 127) // 128)
print(dict(backward_rounds_per_band=int(rounds_sep), backward_rounds_pooled=int(rounds_pool)))
print(dict(backward_pixel_iters_used=int(used), lane_iters_paid_classes=int(paid),
           lane_iters_paid_exact_sort=int(paid_exact), util_classes=round(used / paid, 3),
           util_exact=round(used / paid_exact, 3)))

# adaptive split: within a band-chunk, split the longest items in halves while
# the split items still fit the same number of 64-lane rounds
import heapq  # noqa: E402
paid_split = paid_base = 0
for t, ids in enumerate(tiles):
    ids = sorted(ids)[:256]
    if not ids:
        continue
    ty, tx = divmod(t, tbx)
    ids = np.array(ids)
    X0 = np.maximum(np.ceil(xys[ids, 0] - ex[ids] - 16 * tx), 0)
    X1 = np.minimum(np.floor(xys[ids, 0] + ex[ids] - 16 * tx), 15)
    Y0 = np.maximum(np.ceil(xys[ids, 1] - ey[ids] - 16 * ty), 0)
    Y1 = np.minimum(np.floor(xys[ids, 1] + ey[ids] - 16 * ty), 15)
    ok = (X0 <= X1) & (Y0 <= Y1)
    X0, X1, Y0, Y1 = X0[ok], X1[ok], Y0[ok], Y1[ok]
    for c0 in range(0, len(X0), 64):
        for band in range(2):
            lo, hi = 8 * band, 8 * band + 7
            seq = []
            for e in range(c0, min(c0 + 64, len(X0))):
                r0, r1 = max(Y0[e], lo), min(Y1[e], hi)
                if r0 <= r1:
                    seq += [int(X1[e] - X0[e] + 1)] * int(r1 - r0 + 1)
            if not seq:
                continue
            s = sorted(seq, reverse=True)
            paid_base += sum(64 * s[b] for b in range(0, len(s), 64))
            rounds = (len(s) + 63) // 64
            h = [-x for x in s]
            heapq.heapify(h)
            while len(h) < 64 * rounds and -h[0] > 1:
                x = -heapq.heappop(h)
                heapq.heappush(h, -((x + 1) // 2))
                heapq.heappush(h, -(x // 2))
            s2 = sorted((-x for x in h), reverse=True)
            paid_split += sum(64 * s2[b] for b in range(0, len(s2), 64))
print(dict(exact_sort_paid=int(paid_base), adaptive_split_paid=int(paid_split),
           util_split=round(used / paid_split, 3)))

# the kernel's own form: rows wider than a per-band-chunk brun split in two
# halves (once), brun the smallest (>= 2) that keeps the round count; the
# class layout (4 length classes) as now
def paid_of(items_len):
    cl = classes(np.array(items_len))
    order = np.argsort(-cl, kind="stable")
    s = np.array(items_len)[order]
    return sum(64 * s[b:b + 64].max() for b in range(0, len(s), 64))


paid_now = paid_adapt = 0
for t, ids in enumerate(tiles):
    ids = sorted(ids)[:256]
    if not ids:
        continue
    ty, tx = divmod(t, tbx)
    ids = np.array(ids)
    X0 = np.maximum(np.ceil(xys[ids, 0] - ex[ids] - 16 * tx), 0)
    X1 = np.minimum(np.floor(xys[ids, 0] + ex[ids] - 16 * tx), 15)
    Y0 = np.maximum(np.ceil(xys[ids, 1] - ey[ids] - 16 * ty), 0)
    Y1 = np.minimum(np.floor(xys[ids, 1] + ey[ids] - 16 * ty), 15)
    ok = (X0 <= X1) & (Y0 <= Y1)
    X0, X1, Y0, Y1 = X0[ok], X1[ok], Y0[ok], Y1[ok]
    for c0 in range(0, len(X0), 64):
        for band in range(2):
            lo, hi = 8 * band, 8 * band + 7
            ents = []
            for e in range(c0, min(c0 + 64, len(X0))):
                r0, r1 = max(Y0[e], lo), min(Y1[e], hi)
                if r0 <= r1:
                    ents.append((int(r1 - r0 + 1), int(X1[e] - X0[e] + 1)))
            if not ents:
                continue

            def layout(brun):
                out = []
                for nr, w in ents:  # entry order, an entry's items together
                    out += ([(w + 1) // 2] * 2 if w > brun else [w]) * nr
                return out
            base = layout(16)
            paid_now += paid_of(base)
            rounds = (len(base) + 63) // 64
            best = base
            for brun in range(15, 1, -1):
                cand = layout(brun)
                if (len(cand) + 63) // 64 > rounds:
                    break
                best = cand
            paid_adapt += paid_of(best)
print(dict(paid_now=int(paid_now), paid_adaptive_brun=int(paid_adapt),
           util_now=round(used / paid_now, 3), util_adaptive=round(used / paid_adapt, 3)))
