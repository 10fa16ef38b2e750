"""Train the bench's 1080p / 50k frame (bench.py: seed 1000, target seed 8) on
the GPU for --iters iterations and save it (npz):

* the raw parameters ``_xyz``, ``_cholesky``, ``_features_dc``, ``rgb_W`` --
  the state bench.py's timed steps start from (settle 2000 + warmup 20), the
  input of the trained-density parity fixture (tests/golden/make_golden.py
  ``trained``);
* the activated ``means2d``, ``L``, ``colors`` for offline analysis of the
  trained splat distribution (tile entry counts, rectangle sizes)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2020)
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--gt-seed", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/trained_50k.npz")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    m = make_frame_model(1080, 1920, a.splats, dev, seed=a.seed)
    gt = synthetic_gt(1080, 1920, a.gt_seed, "cpu").to(dev)
    psnr = 0.0
    for it in range(1, a.iters + 1):
        _, psnr = m.train_iter(gt, it)
        if it % 500 == 0:
            print(f"iter {it} psnr {psnr:.4f}", flush=True)
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)

    def np_(t):
        return t.detach().cpu().numpy()

    np.savez_compressed(a.out, _xyz=np_(m._xyz), _cholesky=np_(m._cholesky),
                        _features_dc=np_(m._features_dc), rgb_W=np_(m.rgb_W),
                        means2d=np_(m.get_xyz), L=np_(m.get_cholesky_elements),
                        colors=np_(m.get_features), psnr=psnr, iters=a.iters, seed=a.seed,
                        gt_seed=a.gt_seed)
    print("saved", a.out, "psnr", psnr)


if __name__ == "__main__":
    main()
