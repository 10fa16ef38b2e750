"""Debug: the C++ Function's forward image against the Python Function's (the
diagnostic library's counted binning, knob 0 = 1) on one seeded frame, with
the mismatching pixels' tiles and their entry counts; optional extra knobs for
the Python pass (e.g. 7 1: plain stores) and repeats.

    python tools/op_mismatch.py [--n 50000] [--knob K V] [--repeat 2]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--knob", type=int, nargs=2, action="append", default=[])
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    from conftest import knobs
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    dev = torch.device("cuda:0")
    H, W, n = 1080, 1920, a.n
    g = torch.Generator().manual_seed(n + H)
    means = (2 * torch.rand(n, 2, generator=g) - 1).to(dev)
    L = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5])).to(dev)
    col = torch.rand(n, 3, generator=g).to(dev)
    o = torch.ones(n, 1, device=dev)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    bg = torch.ones(3, device=dev)

    def fwd():
        xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
        return rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, o, H, W, 16, 16,
                                       background=bg), nth

    for r in range(a.repeat):
        fast, nth = fwd()
        with knobs((0, 1), *[tuple(k) for k in a.knob]):
            ref, _ = fwd()
        torch.cuda.synchronize()
        bad = (fast != ref).any(-1)
        ys, xs = torch.nonzero(bad, as_tuple=True)
        tiles = sorted(set(((ys // 16) * tb[0] + xs // 16).tolist()))
        # per-tile entry counts (the projection's bboxes)
        from tile_counts import tile_counts  # noqa: E402
        xys, _, radii, _, _ = project_gaussians_2d(means, L, H, W, tb)
        cnt = tile_counts(xys.detach(), radii, H, W).cpu()
        print(json.dumps(dict(rep=r, bad_pixels=int(bad.sum()), bad_tiles=len(tiles),
                              tiles=tiles[:12], counts=[int(cnt[t]) for t in tiles[:12]],
                              max_count=int(cnt.max()), over256=int((cnt > 256).sum()),
                              over1024=int((cnt > 1024).sum()),
                              maxdiff=float((fast - ref).abs().max()))), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(REPO, "tools"))
    main()
