"""Train the bench's 1080p / 50k frame for --iters iterations on the GPU and
save its parameters (npz) for offline analysis of the trained splat
distribution (tile entry counts, rectangle sizes)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--out", default="gpurun_out/trained_50k.npz")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    m = make_frame_model(1080, 1920, 50000, dev, seed=1000)
    gt = synthetic_gt(1080, 1920, 8, "cpu").to(dev)
    psnr = 0.0
    for it in range(1, a.iters + 1):
        _, psnr = m.train_iter(gt, it)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez_compressed(a.out, means2d=m.get_xyz.detach().cpu().numpy(),
                        L=m.get_cholesky_elements.detach().cpu().numpy(),
                        colors=m.get_features.detach().cpu().numpy(), psnr=psnr)
    print("saved", a.out, "psnr", psnr)


if __name__ == "__main__":
    main()
