"""Debug: one dense trained model (tools/tile_counts.py --save npz) rendered
by every route -- the fused render's first call (density hint 0: id slabs)
and later calls (the hint seen: the banded kernel over record slabs), the op
path without autograd (C++ Function), the Python Function (counted binning,
diagnostic library) -- compared bit for bit; the mismatching pixels' tiles
with their entry counts.

    python tools/render_consistency.py MODEL.npz
    python tools/render_consistency.py CHECKPOINT.pth frame_116   (video driver checkpoint)
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    if sys.argv[1].endswith(".pth"):
        sd = torch.load(sys.argv[1], weights_only=True, map_location="cpu")[sys.argv[2]]
        z = {"xyz": sd["_xyz"].numpy(), "cholesky": sd["_cholesky"].numpy(),
             "features": sd["_features_dc"].numpy()}
    else:
        z = np.load(sys.argv[1])
    from conftest import knobs
    from gsvc_amd.frame import make_frame_model
    from tile_counts import tile_counts
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    n = z["xyz"].shape[0]

    def model(fused_render):
        m = make_frame_model(H, W, n, dev, seed=0, fused_render=fused_render)
        with torch.no_grad():
            m._xyz.copy_(torch.from_numpy(z["xyz"]))
            m._cholesky.copy_(torch.from_numpy(z["cholesky"]))
            m._features_dc.copy_(torch.from_numpy(z["features"]))
        m.eval()
        return m

    outs = {}
    from gsvc_amd import render as R
    with torch.no_grad():
        m = model(True)
        outs["fused_first"] = m()["render"].clone()
        from gsvc_amd.render import render_frame_sum
        bound = torch.tensor([0.5, 0.0, 0.5], device=dev)
        with knobs((0, 2)):  # the banded kernel over record slabs
            outs["banded_records"] = render_frame_sum(m._xyz, m._cholesky, m._features_dc, H, W,
                                                      m.background, cholesky_bound=bound).clone()
        with knobs((24, 1)):  # records at the automatic mode
            outs["records"] = render_frame_sum(m._xyz, m._cholesky, m._features_dc, H, W,
                                               m.background, cholesky_bound=bound).clone()
        for _ in range(30):
            r = m()["render"]
        outs["fused_later"] = r.clone()
        m2 = model(False)
        outs["op_path"] = m2()["render"].clone()
        outs["op_path_2"] = m2()["render"].clone()
        with knobs((0, 1)):
            outs["python_fn"] = m2()["render"].clone()
        from gsvc_amd import ops
        xys, _, radii, _, _ = ops.project_gaussians_2d_forward(
            n, m.get_xyz, m.get_cholesky_elements, H, W, ((W + 15) // 16, (H + 15) // 16, 1), 0.01)
        cnt = tile_counts(xys, radii, H, W).cpu()
    torch.cuda.synchronize()
    ref = outs["python_fn"]
    tbx = (W + 15) // 16
    for k, v in outs.items():
        bad = (v != ref).any(1)[0]
        ys, xs = torch.nonzero(bad, as_tuple=True)
        tiles = sorted(set(((ys // 16) * tbx + xs // 16).tolist()))
        print(json.dumps(dict(route=k, bad_pixels=int(bad.sum()), bad_tiles=len(tiles),
                              counts=sorted([int(cnt[t]) for t in tiles])[-12:],
                              maxdiff=float((v - ref).abs().max()))), flush=True)
    print(json.dumps(dict(max_count=int(cnt.max()), over256=int((cnt > 256).sum()),
                          over1024=int((cnt > 1024).sum()))), flush=True)


if __name__ == "__main__":
    main()
