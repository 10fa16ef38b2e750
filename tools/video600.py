"""BASELINE configs[3] / configs[4] at their defined length on one GPU: the
video driver (gsvc_amd.video, train_video_Represent.py:273-401) over a
600-frame synthetic 1920x1080 video, then a load-back check of the
checkpoint it wrote (gmodels_state_dict.pth, :379,384): every frame's model
is reloaded (torch.load weights_only) into a fresh GaussianVideoFrame, rendered
and scored against its frame; the PSNR must equal the one the driver logged.

    python tools/video600.py --out gpurun_out/v600/c4.json -- \\
        --synthetic 600 --num_points 50000 --iterations 2000 --cut_every 120
    python tools/video600.py --out gpurun_out/v600/c5.json -- \\
        --synthetic 600 --num_points 100000 --iterations 4100 --is_rm --is_ad --cut_every 120

Round 5 adds the harder stand-in: --synthetic_kind textured
(moving, turning textured objects over a mid-frequency background) and
--no_early_stop (fixed iterations per frame).

Writes a summary JSON (wall time, per-frame PSNR / iterations / splat counts,
checkpoint bytes, load-back deviation) to --out; the checkpoint itself (1-2 GB)
stays under --root.  Progress goes to stderr every --every frames.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--root", default="/tmp/gsvc_video600")
    ap.add_argument("--every", type=int, default=25)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    argv = [x for x in a.rest if x != "--"]
    from gsvc_amd import video as V
    from gsvc_amd.frame import GaussianVideoFrame

    vargs = V.parse_args(argv + ["--root", a.root])
    # progress: wrap FrameTrainer.train so every --every frames print a line
    orig_train = V.FrameTrainer.train
    t_start = time.time()
    done = [0]

    def train_logged(self):
        r = orig_train(self)
        done[0] += 1
        if done[0] % a.every == 0 or done[0] == 1:
            print(f"[video600] frame {self.frame_num}: psnr {r['psnr']:.3f} it {r['iterations']} "
                  f"n {r['num_gaussians']} train {r['training_time']:.3f}s "
                  f"elapsed {time.time() - t_start:.0f}s", file=sys.stderr, flush=True)
        return r

    V.FrameTrainer.train = train_logged
    t0 = time.time()
    res = V.main(argv + ["--root", a.root])
    wall = time.time() - t0
    frames = res["frames"]
    mdir = (os.path.join(a.root, vargs.savdir_m, vargs.data_name,
                         f"{vargs.model_name}_{vargs.iterations}_{vargs.num_points}"))
    ckpt = os.path.join(mdir, "gmodels_state_dict.pth")
    ckpt_bytes = os.path.getsize(ckpt)

    # load-back: every frame's model from the checkpoint, rendered and scored
    dev = torch.device("cuda:0")
    t1 = time.time()
    models = torch.load(ckpt, weights_only=True, map_location="cpu")
    make = V.textured_video if vargs.synthetic_kind == "textured" else V.synthetic_video
    gen = make(vargs.synthetic, vargs.height, vargs.width, int(vargs.seed), vargs.cut_every, device=dev)
    dev_psnr = []
    for r in frames:
        f = r["frame"]
        sd = models[f"frame_{f}"]
        n = sd["_xyz"].shape[0]
        m = GaussianVideoFrame(loss_type="L2", opt_type="adan", num_points=n, max_num_points=n,
                               densification_interval=100, iterations=1, H=vargs.height,
                               W=vargs.width, BLOCK_H=16, BLOCK_W=16, device=dev, lr=1e-3,
                               quantize=False, removal_rate=0.1, isdensity=False,
                               isremoval=False).to(dev)
        full = m.state_dict()
        full.update({k: v.to(dev) for k, v in sd.items()})
        m.load_state_dict(full)
        m.eval()
        with torch.no_grad():
            out = m()["render"]
            mse = float(F.mse_loss(out, gen(f - 1)))
        p = 10 * math.log10(1.0 / mse)
        dev_psnr.append(abs(p - r["psnr"]))
    reload_s = time.time() - t1
    psnrs = [r["psnr"] for r in frames]
    summary = dict(
        argv=argv, frames=len(frames), wall_s=round(wall, 2), reload_s=round(reload_s, 2),
        k_frames=sorted({r["frame"] for r in frames if r["frame"] in set(_k(mdir, a.root, vargs))}),
        avg_psnr=sum(psnrs) / len(psnrs), min_psnr=min(psnrs), max_psnr=max(psnrs),
        avg_ms_ssim=res["average"]["ms_ssim"],
        total_training_s=sum(r["training_time"] for r in frames),
        total_iterations=sum(r["iterations"] for r in frames),
        train_iters_per_s=sum(r["iterations"] for r in frames) / sum(r["training_time"] for r in frames),
        avg_eval_fps=res["average"]["eval_fps"],
        splats_min=min(r["num_gaussians"] for r in frames),
        splats_max=max(r["num_gaussians"] for r in frames),
        checkpoint_bytes=ckpt_bytes, checkpoint_frames=len(models),
        reload_max_abs_psnr_diff=max(dev_psnr),
        per_frame=[dict(frame=r["frame"], psnr=round(r["psnr"], 5), ms_ssim=r["ms_ssim"],
                        iterations=r["iterations"], splats=r["num_gaussians"],
                        train_s=round(r["training_time"], 4), eval_fps=round(r["eval_fps"], 1),
                        reload_dpsnr=d)
                   for r, d in zip(frames, dev_psnr)])
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "per_frame"}), flush=True)
    if summary["checkpoint_frames"] != summary["frames"] or max(dev_psnr) > 1e-6:
        raise SystemExit("video600: checkpoint load-back mismatch")


def _k(mdir, root, vargs):
    p = os.path.join(root, vargs.savdir, vargs.data_name, "K_frames_used.txt")
    try:
        with open(p) as fh:
            return [int(x) for x in fh.read().split()]
    except OSError:
        return []


if __name__ == "__main__":
    main()
