"""Dump the first 4096 splats' parameters after the reference trajectory's
iterations (fused and op-by-op paths) for offline comparison with
tests/golden/train_traj_1080p_n50k.npz."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gsvc_amd.frame import make_frame_model, synthetic_gt  # noqa: E402

z = np.load(os.path.join(REPO, "tests/golden/train_traj_1080p_n50k.npz"))
dev = torch.device("cuda:0")
out = {}
for fused in (True, False):
    iters = int(z["iters"]) if fused else int(sys.argv[1]) if len(sys.argv) > 1 else 40
    m = make_frame_model(int(z["H"]), int(z["W"]), int(z["n"]), dev, seed=int(z["seed"]),
                         fused_train=fused)
    gt = synthetic_gt(int(z["H"]), int(z["W"]), int(z["gt_seed"]), "cpu").to(dev)
    ps = []
    for it in range(1, iters + 1):
        _, p = m.train_iter(gt, it)
        ps.append(p)
    tag = "fused" if fused else "op"
    out[tag + "_psnrs"] = np.array(ps)
    for k in ("_xyz", "_cholesky", "_features_dc"):
        out[f"{tag}_{k}"] = getattr(m, k).detach().cpu().numpy()[:4096]
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "traj_dump.npz"), **out)
print("ok")
