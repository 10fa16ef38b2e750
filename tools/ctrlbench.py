"""Cost of the prune / densify iterations (GaussianSplats_Represent.py:98-172)
next to the fused ones: per-iteration wall time of GaussianVideoFrame.train_iter
at 1920x1080 with removal (K-frame style) or densification (P-frame style)
every --interval iterations.

    python tools/ctrlbench.py [--splats 100000] [--iters 600] [--interval 100]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, default=100000)
    ap.add_argument("--iters", type=int, default=600)
    ap.add_argument("--interval", type=int, default=100)
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    gt = synthetic_gt(H, W, 8, dev)
    for mode in ("removal", "densify"):
        model = make_frame_model(H, W, a.splats, dev, seed=7, isremoval=mode == "removal",
                                 isdensity=mode == "densify", removal_rate=0.1,
                                 max_num_points=a.splats, densification_interval=a.interval)
        ctrl, plain = [], []
        for it in range(1, a.iters + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model.train_iter(gt, it)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e6
            is_ctrl = (it == 1 and mode == "densify") or it % a.interval == 0
            (ctrl if is_ctrl else plain).append(dt)
        plain.sort()
        print(json.dumps(dict(mode=mode, splats_end=int(model._xyz.shape[0]),
                              control_iters=len(ctrl), control_us=[round(x) for x in ctrl],
                              plain_median_us=round(plain[len(plain) // 2], 1),
                              amortized_control_us_per_iter=round(sum(ctrl) / a.iters, 1))),
              flush=True)


if __name__ == "__main__":
    main()
