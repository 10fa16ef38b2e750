"""Host cost of one fused train_iter: a 16x16 / 16-splat model (no GPU
back-pressure), per iteration, with a cProfile of the Python side.

    python tools/trainhost.py [--iters 2000] [--profile]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    m = make_frame_model(16, 16, 16, dev, seed=3)
    gt = synthetic_gt(16, 16, 1, dev)
    for it in range(1, 51):
        m.train_iter(gt, it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(51, 51 + a.iters):
        m.train_iter(gt, it)
    dt = (time.perf_counter() - t0) / a.iters * 1e6
    print(json.dumps(dict(host_us_per_iter=round(dt, 2), fused_steps=m.fused_steps)), flush=True)
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        for it in range(51 + a.iters, 51 + 2 * a.iters):
            m.train_iter(gt, it)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
        print(s.getvalue()[:4000])


if __name__ == "__main__":
    main()
