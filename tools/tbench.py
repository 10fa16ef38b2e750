"""Training-iteration microbenchmark: GaussianVideoFrame.train_iter at
1920x1080 (BASELINE configs[2]: 50k splats by default), iterations/s.
Run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.

    python tools/tbench.py [--splats 50000] [--iters 100] [--foreach-adan]
"""
from __future__ import annotations

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
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--foreach-adan", action="store_true")
    ap.add_argument("--op-by-op", action="store_true", help="disable the fused training step")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    model = make_frame_model(H, W, a.splats, dev, seed=7,
                             fused_adan=False if a.foreach_adan else None,
                             fused_train=False if a.op_by_op else None)
    gt = synthetic_gt(H, W, 8, dev)
    for it in range(1, a.warmup + 1):
        model.train_iter(gt, it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    psnr = 0.0
    for it in range(a.warmup + 1, a.warmup + a.iters + 1):
        _, psnr = model.train_iter(gt, it)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(json.dumps(dict(splats=a.splats, fused_adan=model.fused_adan,
                          fused_train=model.fused_steps > 0, iters_per_s=round(1 / dt, 1),
                          ms_per_iter=round(1e3 * dt, 4), psnr=round(psnr, 3))), flush=True)


if __name__ == "__main__":
    main()
