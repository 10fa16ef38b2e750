"""Workloads of bench.py for rocprofv3 kernel-trace / PMC passes (run under
``rocprofv3 ... -- python3 tools/pmc_workloads.py MODE``):

  train50k   GaussianVideoFrame at 1920x1080 / 50k splats: --settle training
             iterations, then --iters more (the bench's trained state), then
             --iters renders of the trained model (configs[2] render);
  render10k  --iters renders of a random-init 10k-splat frame (configs[1]).

Summaries take each kernel's last --iters dispatches (tools/prof_summary.py
--last), i.e. the trained state.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["train50k", "render10k"])
    ap.add_argument("--settle", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    if a.mode == "train50k":
        model = make_frame_model(H, W, 50000, dev, seed=1000)
        gt = synthetic_gt(H, W, 8, "cpu").to(dev)
        for it in range(1, a.settle + a.iters + 1):
            model.train_iter(gt, it)
        model.eval()
    else:
        model = make_frame_model(H, W, 10000, dev, seed=1000)
        model.eval()
    with torch.no_grad():
        for _ in range(a.iters):
            model()
    torch.cuda.synchronize()
    print("done", a.mode, flush=True)


if __name__ == "__main__":
    main()
