"""Timing of SSIM / MS-SSIM at 1920x1080x3 (the loss and the per-frame metric):
the gfx950 kernels (gsvc_amd.msssim) next to a torch restatement of
pytorch_msssim on the same GPU (F.conv2d grouped windows + F.avg_pool2d,
tests/test_ssim.py), forward and forward+backward, HIP events over --iters calls.

    python tools/ssimbench.py [--iters 50]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402

from gsvc_amd.msssim import ms_ssim, ssim  # noqa: E402
from test_ssim import t_ms_ssim, t_ssim  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only-hip", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.rand((1, 3, 1080, 1920), device=dev, generator=g)
    Y = (X + 0.1 * torch.randn(X.shape, device=dev, generator=g)).clamp(0, 1)
    impls = [("hip", ssim, ms_ssim)] + ([] if args.only_hip else [("torch", t_ssim, t_ms_ssim)])
    for name, f_ssim, f_ms in impls:
        for label, f in (("ssim", lambda x: f_ssim(x, Y, data_range=1)),
                         ("ms_ssim", lambda x: f_ms(x, Y, data_range=1))):
            fwd = timed(lambda: f(X), args.iters)
            xr = X.clone().requires_grad_(True)

            def fb():
                xr.grad = None
                f(xr).backward()
            both = timed(fb, args.iters)
            print(json.dumps(dict(impl=name, op=label, H=1080, W=1920, C=3,
                                  fwd_us=round(fwd, 1), fwd_bwd_us=round(both, 1))), flush=True)


if __name__ == "__main__":
    main()
