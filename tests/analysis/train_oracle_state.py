"""Train bench.py's 1080p / 50k frame (seed 1000, target seed 8) on the CPU
with the oracle's train_iter_sum (oracle/oracle.py: the C restatement of the
reference kernels + the reference's L2 / Adan glue, OpenMP over tiles) for
--iters iterations and save the raw parameters -- the settled, trained-density
state that tests/golden/make_golden.py ``trained`` turns into the parity
fixture of the state bench.py times.  Test
infrastructure: build container only."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2020)
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--gt-seed", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/trained_cpu/state_50k_s1000.npz")
    a = ap.parse_args()
    import oracle as O
    from gsvc_amd.frame import synthetic_gt
    O.set_threads(a.threads)
    n = a.splats
    g = torch.Generator().manual_seed(a.seed)  # GaussianSplats_Represent.py:28-38 draw order
    params = dict(_xyz=torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5)).numpy(),
                  _cholesky=torch.rand(n, 3, generator=g).numpy(),
                  _features_dc=torch.rand(n, 3, generator=g).numpy())
    gt = synthetic_gt(1080, 1920, a.gt_seed, "cpu").numpy()[0]
    state = {}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    t0 = time.time()
    psnr = 0.0
    for it in range(1, a.iters + 1):
        _, psnr = O.train_iter_sum(params, gt, 1080, 1920, state, it)
        if it % 50 == 0:
            print(f"iter {it} psnr {psnr:.4f} {time.time() - t0:.0f}s", flush=True)
    np.savez_compressed(a.out, _xyz=params["_xyz"], _cholesky=params["_cholesky"],
                        _features_dc=params["_features_dc"], rgb_W=np.ones((n, 1), np.float32),
                        psnr=psnr, iters=a.iters, seed=a.seed, gt_seed=a.gt_seed)
    print("saved", a.out, "psnr", psnr, f"{time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
