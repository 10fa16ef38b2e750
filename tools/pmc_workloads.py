"""Workloads of bench.py for rocprofv3 kernel-trace / PMC passes (run under
``rocprofv3 ... -- python3 tools/pmc_workloads.py MODE``):

  train50k   GaussianVideoFrame at 1920x1080 / 50k splats: --settle training
             iterations, then --iters more (the bench's trained state), then
             --warm + --iters renders of the trained model (configs[2] render);
  render10k  --warm + --iters renders of a random-init 10k-splat frame (configs[1]);
  decode8    --iters batched renders of a GOP of 8 distinct 10k-splat frame
             models (bench.py ``video_decode``: one gsvc_render_frames_sum call);
  oppath     train50k's trained state, then --iters forward + backward calls of
             the unchanged-caller op path (bench.py ``op_path``);
  alpha50k   --iters forward + backward calls of the alpha operators at 1080p /
             50k, opacity U(0.1, 1) (bench.py ``alpha``).

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
    ap.add_argument("mode", choices=["train50k", "render10k", "decode8", "oppath", "alpha50k"])
    ap.add_argument("--settle", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warm", type=int, default=200,
                    help="renders before the --iters summarised ones (bench.py times its renders "
                         "after warm-up; the first calls include the unordered projection and a "
                         "cold clock)")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    H, W = 1080, 1920
    if a.mode == "decode8":
        from gsvc_amd.render import render_frames_sum
        frames, splats = 8, 10000
        g = torch.Generator().manual_seed(4242)  # bench.py video_decode's inputs
        xyz = torch.atanh(2 * (torch.rand(frames * splats, 2, generator=g) - 0.5)).to(dev)
        chol = torch.rand(frames * splats, 3, generator=g).to(dev)
        feat = torch.rand(frames * splats, 3, generator=g).to(dev)
        bound = torch.tensor([0.5, 0.0, 0.5], device=dev)
        bg = torch.ones(3, device=dev)
        for _ in range(a.iters + 5):
            render_frames_sum(xyz, chol, feat, [splats] * frames, H, W, bg, cholesky_bound=bound)
        torch.cuda.synchronize()
        print("done", a.mode, flush=True)
        return
    if a.mode == "alpha50k":
        from gsplat.project_gaussians_2d import project_gaussians_2d
        from gsplat.rasterize import rasterize_gaussians
        n = 50000
        g = torch.Generator().manual_seed(n)  # bench.py alpha_block's inputs
        ps = [torch.tanh(torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5))),
              torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5]),
              torch.rand(n, 3, generator=g), 0.1 + 0.9 * torch.rand(n, 1, generator=g)]
        ps = [p.to(dev).requires_grad_(True) for p in ps]
        bg = torch.ones(3, device=dev)
        tb = ((W + 15) // 16, (H + 15) // 16, 1)
        for _ in range(a.iters + 5):
            xys, depths, radii, conics, nth = project_gaussians_2d(ps[0], ps[1], H, W, tb)
            out = rasterize_gaussians(xys, depths, radii, conics, nth, ps[2], ps[3], H, W, 16, 16,
                                      background=bg)
            torch.autograd.grad(out.sum(), ps)
        torch.cuda.synchronize()
        print("done", a.mode, flush=True)
        return
    if a.mode in ("train50k", "oppath"):
        model = make_frame_model(H, W, 50000, dev, seed=1000)
        gt = synthetic_gt(H, W, 8, "cpu").to(dev)
        for it in range(1, a.settle + a.iters + 1):
            model.train_iter(gt, it)
        model.eval()
        if a.mode == "oppath":  # GSVC's own op sequence over the drop-in, on the trained frame
            import torch.nn.functional as F
            op = make_frame_model(H, W, 50000, dev, seed=0, fused_train=False, fused_render=False)
            with torch.no_grad():
                for k in ("_xyz", "_cholesky", "_features_dc"):
                    getattr(op, k).copy_(getattr(model, k))
            for _ in range(a.iters + 5):
                img = op.forward()["render"]
                F.mse_loss(img.squeeze(0), gt.squeeze(0)).backward()
            torch.cuda.synchronize()
            print("done", a.mode, flush=True)
            return
    else:
        model = make_frame_model(H, W, 10000, dev, seed=1000)
        model.eval()
    with torch.no_grad():
        for _ in range(a.warm + a.iters):
            model()
    torch.cuda.synchronize()
    print("done", a.mode, flush=True)


if __name__ == "__main__":
    main()
