"""GSVC's video driver on the gsvc_amd hot path, sharded by GOP across GPUs.

A restatement of train_video_Represent.py (reference :17-401) and the helpers
it uses from utils.py (process_yuv_video :134-156, EarlyStopping :188-211,
detect_outliers_mean_diff :214-229) that runs on the MI355X path:

* frames come from a planar I420 file (converted on the GPU by
  ``gsvc_i420_to_rgb``, OpenCV's BT.601 arithmetic) or from a seeded synthetic
  video (the UVG sequences are not in this image);
* K-frames (key frames, trained from scratch) come from
  ``<savdir>/<data>/K_frames.txt`` when present, else from the reference's
  detector (500 scratch iterations and a 100-iteration P-probe per frame,
  normalised loss differences, mean-difference outliers), run with every
  rank taking a contiguous frame range plus a one-frame halo;
* the frames are split into GOPs (a K-frame and the P-frames after it, which
  start from the previous frame's model) and ranks take contiguous GOPs
  (shard.py); when there are fewer GOPs than ranks, K-frames are forced at
  the shard boundaries; K_frames_used.txt records the GOPs trained and a
  missing K_frames.txt is written from detection (never overwritten);
* each frame trains with ``GaussianVideoFrame.train_iter`` (the fused step on
  the GPU), early stopping as the reference, then PSNR and the eval FPS of
  100 renders (synchronised);
* the per-frame metrics meet in ONE all_reduce (RCCL over xGMI with the
  "nccl" backend; gloo on CPU), the only collective of the path;
* ``--ranks_per_gpu R`` puts R ranks (R GOP shards) on each GPU: one frame's
  step leaves part of the chip idle, so two concurrent shards train ~1.35x as
  many iterations per second; their collectives go over gloo.

    python -m gsvc_amd.video --synthetic 24 --width 256 --height 256 --num_points 2000 \\
        --iterations 300 --loss_type L2
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m gsvc_amd.video -d Beauty.yuv ...

The per-frame MS-SSIM is gsvc_amd.msssim.ms_ssim (pytorch_msssim's algorithm
on the gfx950 kernels; parity unpinned against the package);
frames whose smaller side is <= 160 (where ms_ssim asserts) report NaN.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .frame import GaussianVideoFrame
from .msssim import ms_ssim
from .shard import aggregate_video_metrics, forced_k_frames, gops, shard_gops

# ---------------------------------------------------------------------------
# frames


def i420_to_rgb(yuv: torch.Tensor, height: int, width: int) -> torch.Tensor:
    """One I420 frame (uint8 device tensor) -> [1, 3, H, W] float RGB in [0, 1]
    (cv2.cvtColor(COLOR_YUV2RGB_I420) + ToTensor) on the GPU."""
    from . import _lib as L
    if not yuv.is_cuda or yuv.dtype != torch.uint8:
        raise RuntimeError("yuv must be a uint8 CUDA tensor")
    if yuv.numel() != height * width * 3 // 2:
        raise ValueError("yuv must hold one I420 frame of H*W*3/2 bytes")
    out = torch.empty((1, 3, height, width), dtype=torch.float32, device=yuv.device)
    L.call("gsvc_i420_to_rgb", L.ptr(yuv.contiguous()), int(height), int(width), L.ptr(out),
           L.stream(yuv.device))
    return out


def load_yuv_frames(path: str, width: int, height: int, device, frames: Optional[Sequence[int]] = None):
    """process_yuv_video (utils.py:134-156) for the 0-based frame indices
    ``frames`` (all when None): a memory map, one frame at a time to the GPU."""
    size = width * height * 3 // 2
    total = os.path.getsize(path) // size
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    idx = range(total) if frames is None else frames
    out = {}
    for i in idx:
        if not 0 <= i < total:
            continue
        raw = torch.from_numpy(np.array(mm[i * size:(i + 1) * size])).to(device)
        out[i] = i420_to_rgb(raw, height, width)
    return out, total


def textured_video(num_frames: int, height: int, width: int, seed: int = 0, cut_every: int = 0,
                   device=None, objects: int = 14):
    """A harder stand-in for the UVG sequences: per scene a
    mid-frequency background (drifting sinusoids up to ~30 cycles across the
    frame) under ``objects`` hard-edged elliptical objects, each with its own
    striped / checkered texture (periods 6-24 px) and colours, moving (2-9 px
    per frame) and turning from frame to frame, drawn back to front; a scene
    cut every ``cut_every`` frames.  Sharp edges, texture and motion keep the
    per-frame models training (the smooth pattern of ``synthetic_video``
    converges in a few hundred iterations).  Computed with torch on ``device``
    (CPU by default); frame(i) -> [1, 3, H, W] in [0, 1]."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    yy, xx = torch.meshgrid(torch.arange(height, device=dev, dtype=torch.float32),
                            torch.arange(width, device=dev, dtype=torch.float32), indexing="ij")
    diag = float(np.hypot(height, width))

    def frame(i: int) -> torch.Tensor:
        scene = i // cut_every if cut_every else 0
        t = float(i - (scene * cut_every if cut_every else 0))
        rng = np.random.default_rng(seed * 7919 + scene * 104729 + 17)
        img = []
        bg = rng.uniform(0, 1, (3, 4, 5))
        for c in range(3):
            acc = torch.zeros((height, width), device=dev)
            for k in range(4):
                fx, fy, ph, vx, vy = (float(v) for v in bg[c, k])
                acc += torch.sin((60 * fx * xx + 60 * fy * yy) / diag * 3.0 +
                                 6.28 * ph + 0.15 * t * (vx - vy))
            img.append(0.5 + 0.35 * acc / 4)
        img = torch.stack(img)
        for _ in range(objects):
            cx, cy = rng.uniform(0, width), rng.uniform(0, height)
            rx, ry = rng.uniform(40, 260), rng.uniform(40, 260)
            ang, w = rng.uniform(0, np.pi), rng.uniform(-0.03, 0.03)
            vx, vy = rng.uniform(-9, 9), rng.uniform(-6, 6)
            period = rng.uniform(6, 24)
            kind = rng.integers(0, 2)
            c1, c2 = rng.uniform(0, 1, 3), rng.uniform(0, 1, 3)
            ox, oy = cx + vx * t, cy + vy * t
            a = ang + w * t
            ca, sa = float(np.cos(a)), float(np.sin(a))
            u = (xx - ox) * ca + (yy - oy) * sa
            v = -(xx - ox) * sa + (yy - oy) * ca
            inside = (u / rx) ** 2 + (v / ry) ** 2 <= 1.0
            if kind == 0:  # stripes
                pat = (torch.floor(u / period) % 2) == 0
            else:  # checks
                pat = ((torch.floor(u / period) + torch.floor(v / period)) % 2) == 0
            for ch in range(3):
                col = torch.where(pat, torch.tensor(float(c1[ch]), device=dev),
                                  torch.tensor(float(c2[ch]), device=dev))
                img[ch] = torch.where(inside, col, img[ch])
        return img.clamp(0, 1)[None].contiguous()

    return frame


def synthetic_video(num_frames: int, height: int, width: int, seed: int = 0, cut_every: int = 0,
                    device=None):
    """A seeded smooth moving RGB pattern (sum of drifting sinusoids per
    channel), with a scene cut (new pattern) every ``cut_every`` frames: the
    stand-in for the UVG sequences.  Returns a function frame(i) -> [1, 3, H, W]
    in [0, 1] so ranks materialise only their own frames: on the CPU (numpy)
    by default, or computed on ``device`` with torch (a 1080p frame is ~36 M
    sines: ~0.3 s on one host core, microseconds on the GPU; the two agree to
    float32 rounding of sin)."""
    if device is not None and torch.device(device).type != "cpu":
        dev = torch.device(device)
        yy_t, xx_t = torch.meshgrid(torch.linspace(0, 1, height, device=dev),
                                    torch.linspace(0, 1, width, device=dev), indexing="ij")

        def frame_dev(i: int) -> torch.Tensor:
            scene = i // cut_every if cut_every else 0
            rng = np.random.default_rng(seed * 1000003 + scene)
            par = rng.uniform(0, 1, (3, 6, 5)).astype(np.float32)
            t = np.float32(i - (scene * cut_every if cut_every else 0))
            chans = []
            for c in range(3):
                acc = torch.zeros((height, width), device=dev)
                for k in range(6):
                    fx, fy, ph, vx, vy = (float(v) for v in par[c, k])
                    acc += torch.sin(12 * fx * xx_t + 12 * fy * yy_t +
                                     (6.28 * ph + float(0.08 * t * (vx + vy))))
                chans.append(0.5 + 0.5 * acc / 6)
            return torch.stack(chans).clamp(0, 1)[None].contiguous()

        return frame_dev
    yy, xx = np.meshgrid(np.linspace(0, 1, height, dtype=np.float32),
                         np.linspace(0, 1, width, dtype=np.float32), indexing="ij")

    def frame(i: int) -> torch.Tensor:
        scene = i // cut_every if cut_every else 0
        rng = np.random.default_rng(seed * 1000003 + scene)
        par = rng.uniform(0, 1, (3, 6, 5)).astype(np.float32)
        t = np.float32(i - (scene * cut_every if cut_every else 0))
        chans = []
        for c in range(3):
            acc = np.zeros((height, width), np.float32)
            for k in range(6):
                fx, fy, ph, vx, vy = par[c, k]
                acc += np.sin(12 * fx * xx + 12 * fy * yy + 6.28 * ph + 0.08 * t * (vx + vy))
            chans.append(0.5 + 0.5 * acc / 6)
        return torch.from_numpy(np.clip(np.stack(chans), 0, 1)[None].astype(np.float32))

    return frame


# ---------------------------------------------------------------------------
# reference helpers (utils.py:188-229)


class EarlyStopping:
    """The convergence test of train_video_Represent.py:79-96 (reference
    utils.py:188-211): stop once ``patience`` consecutive losses have failed to
    beat the best loss so far by more than ``min_delta``; the first loss only
    sets the best."""

    def __init__(self, patience=100, min_delta=0.0):
        self.patience, self.min_delta = patience, min_delta
        self.best_loss = None
        self.counter = 0

    def __call__(self, current_loss) -> bool:
        stale = self.best_loss is not None and not (self.best_loss - current_loss > self.min_delta)
        if stale:
            self.counter += 1
            return self.counter >= self.patience
        first = self.best_loss is None
        self.best_loss, self.counter = current_loss, 0
        return (not first) and self.patience <= 0


def detect_outliers_mean_diff(values, window_size=10, threshold=3):
    """K-frame candidates of train_video_Represent.py:348-353 (reference
    utils.py:214-229): index i is an outlier when it exceeds the mean of its
    window [i - window_size, i + window_size) (clipped to the sequence) by more
    than ``threshold`` population standard deviations of that window, or is
    more than ``threshold`` times that mean."""
    v = np.asarray(values, dtype=np.float64)
    n = len(v)
    lo = np.maximum(np.arange(n) - window_size, 0)
    hi = np.minimum(np.arange(n) + window_size, n)
    stats = np.array([(np.mean(v[a:b]), np.std(v[a:b])) for a, b in zip(lo, hi)]).reshape(n, 2)
    mean, std = stats[:, 0], stats[:, 1]
    hit = ((v - mean) > threshold * std) | (v > mean * threshold)
    return [int(i) for i in np.flatnonzero(hit)]


# ---------------------------------------------------------------------------
# per-frame trainer (SimpleTrainer2d, train_video_Represent.py:17-202)


class FrameTrainer:
    def __init__(self, image: torch.Tensor, frame_num: int, loss_type: str = "L2",
                 num_points: int = 2000, max_num_points: int = 2000, iterations: int = 30000,
                 lr: float = 1e-3, densification_interval: int = 100, trained_model=None,
                 isdensity=False, isremoval=True, removal_rate=0.25, early_stop=True):
        self.device = image.device
        self.early_stop = early_stop  # False: every frame trains for ``iterations``
        self.gt_image = image
        self.frame_num = frame_num
        self.iterations = iterations
        self.isdensity, self.isremoval = isdensity, isremoval
        self.H, self.W = image.shape[2], image.shape[3]
        self.model = GaussianVideoFrame(
            loss_type=loss_type, opt_type="adan", num_points=num_points,
            max_num_points=max_num_points, densification_interval=densification_interval,
            iterations=iterations, H=self.H, W=self.W, BLOCK_H=16, BLOCK_W=16, device=self.device,
            lr=lr, quantize=False, removal_rate=removal_rate, isdensity=isdensity,
            isremoval=isremoval).to(self.device)
        if trained_model is not None:  # :64-69, partial load
            sd = self.model.state_dict()
            sd.update({k: v for k, v in trained_model.items() if k in sd})
            self.model.load_state_dict(sd)

    def _filtered(self):
        sd = self.model.state_dict()
        out = {k: sd[k].detach().clone() for k in ("_xyz", "_cholesky")}
        out["_features_dc"] = self.model.get_features.detach().clone()
        return out

    def pre_train(self):
        """:117-133 (the K-frame detector's probe): no early stopping."""
        self.model.train()
        loss = None
        for it in range(1, int(self.iterations) + 1):
            loss, _ = self.model.pre_train_iter(self.gt_image)
        return self._filtered(), float(loss)

    def train(self):
        """:79-114: train with early stopping, then PSNR and eval FPS."""
        self.model.train()
        t0 = time.time()
        early = EarlyStopping(patience=100, min_delta=1e-9)
        stable = 5000
        loss = None
        it = 0
        for it in range(1, int(self.iterations) + 1):
            loss, psnr = self.model.train_iter(self.gt_image, it)
            if not self.early_stop:
                continue
            lv = float(loss.detach())
            if self.isdensity or self.isremoval:
                stable -= 1
                if stable < 0 and early(lv):
                    break
            elif early(lv):
                break
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        train_time = time.time() - t0
        self.model.eval()
        with torch.no_grad():
            out = self.model()["render"]
            mse = F.mse_loss(out.float(), self.gt_image.float())
            psnr = 10 * math.log10(1.0 / float(mse))
            # :145; ms_ssim needs a smaller side > 160 (the reference asserts):
            # smaller frames report NaN
            ms = float("nan")
            if min(self.H, self.W) > 160 and self.device.type == "cuda":
                ms = float(ms_ssim(out.float(), self.gt_image.float(), data_range=1,
                                   size_average=True))
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            t1 = time.time()
            for _ in range(100):
                self.model()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            eval_time = (time.time() - t1) / 100
        return dict(psnr=psnr, ms_ssim=ms, training_time=train_time,
                    eval_time=eval_time, eval_fps=1.0 / eval_time,
                    num_gaussians=int(self.model._xyz.shape[0]), loss=float(loss.detach()),
                    iterations=it, model=self._filtered())


# ---------------------------------------------------------------------------
# K-frames and the sharded video loop


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def detect_k_frames(frame_fn, num_frames: int, rank: int, world: int, loss_type: str, lr: float,
                    probe_points=5000, scratch_iters=500, probe_iters=100, seed: int = 1) -> List[int]:
    """train_video_Represent.py:318-355 with frames split over ranks: rank r
    probes a contiguous range and recomputes the scratch model of the frame
    before its range (one-frame halo); the normalised loss list is gathered
    so that every rank finds the same outliers."""
    lo, hi = (num_frames * rank) // world, (num_frames * (rank + 1)) // world
    losses: Dict[int, float] = {}
    prev = None
    for i in range(max(lo - 1, 0), hi):
        img = frame_fn(i)
        # seeded by frame, not by rank: the halo frame's scratch model is the one
        # its owner trains, and the list does not depend on the world size
        torch.manual_seed(seed + i)
        k = FrameTrainer(img, i + 1, loss_type, probe_points, probe_points, scratch_iters, lr,
                         isdensity=False, isremoval=False)
        gm, loss_k = k.pre_train()
        if i >= lo:
            if i == 0:
                losses[i] = 0.0
            else:
                p = FrameTrainer(img, i + 1, loss_type, probe_points, probe_points, probe_iters, lr,
                                 trained_model=prev, isdensity=False, isremoval=False)
                _, loss_p = p.pre_train()
                losses[i] = loss_p - loss_k
        prev = gm
    d = _dist()
    if d is not None:
        parts = [None] * world
        d.all_gather_object(parts, losses)
        for part in parts:
            losses.update(part)
    vals = np.array([losses[i] for i in range(num_frames)], np.float64)
    rest = vals[1:]
    if len(rest):
        mn, mx = rest.min(), rest.max()
        span = (mx - mn) if mx > mn else 1.0
        norm = [vals[0]] + [(v - mn) / span for v in rest]
    else:
        norm = [vals[0]]
    ks = [int(x + 1) for x in detect_outliers_mean_diff(norm)]
    return sorted(set([1] + ks))


def train_video(frame_fn, num_frames: int, k_frames: Sequence[int], args, rank: int, world: int,
                device) -> Dict:
    """The per-frame loop of train_video_Represent.py:358-398 over this rank's
    GOPs; returns the video-wide averages (one all_reduce) and this rank's
    per-frame log and models."""
    shards = shard_gops(k_frames, num_frames, world)
    mine = shards[rank]
    per = {k: [] for k in ("psnr", "ms_ssim", "training_time", "eval_time", "eval_fps",
                           "num_gaussians")}
    log, models = [], {}
    for start, end in mine:
        gmodel, npts = None, args.num_points
        for f in range(start, end):  # 1-based frame numbers
            img = frame_fn(f - 1).to(device)
            # seeded by frame: a frame's init is the same on any number of ranks
            torch.manual_seed(int(getattr(args, "seed", 1)) + f)
            if f == start:  # a K-frame: from scratch
                tr = FrameTrainer(img, f, args.loss_type, args.num_points, args.num_points,
                                  args.iterations, args.lr, args.densification_interval,
                                  isdensity=False, isremoval=args.is_rm,
                                  removal_rate=args.removal_rate,
                                  early_stop=not getattr(args, "no_early_stop", False))
            else:  # a P-frame: from the previous frame's model
                tr = FrameTrainer(img, f, args.loss_type, npts, args.num_points, args.iterations,
                                  args.lr, args.densification_interval, trained_model=gmodel,
                                  isdensity=args.is_ad, isremoval=False,
                                  removal_rate=args.removal_rate,
                                  early_stop=not getattr(args, "no_early_stop", False))
            r = tr.train()
            gmodel, npts = r.pop("model"), r["num_gaussians"]
            models[f"frame_{f}"] = {k: v.cpu() for k, v in gmodel.items()}
            for k in per:
                per[k].append(r[k])
            log.append(dict(frame=f, **{k: r[k] for k in r}))
    avg = aggregate_video_metrics(per, device=device if getattr(args, "backend", "") == "nccl"
                                  else None)
    return dict(average=avg, frames=log, models=models, gops=[list(g) for g in mine])


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="GSVC video representation on MI355X")
    ap.add_argument("-d", "--dataset", type=str, default=None, help="I420 .yuv file")
    ap.add_argument("--synthetic", type=int, default=0, help="frames of a synthetic video")
    ap.add_argument("--cut_every", type=int, default=0, help="synthetic scene-cut period")
    ap.add_argument("--synthetic_kind", choices=["smooth", "textured"], default="smooth",
                    help="smooth drifting sinusoids, or textured moving objects (harder)")
    ap.add_argument("--no_early_stop", action="store_true",
                    help="train every frame for --iterations (SURVEY 8d config 4: fixed "
                         "iterations per frame, early stopping off)")
    ap.add_argument("--data_name", type=str, default="Synthetic")
    ap.add_argument("--model_name", type=str, default="GaussianVideo")
    ap.add_argument("--savdir", type=str, default="result")
    ap.add_argument("--savdir_m", type=str, default="models")
    ap.add_argument("--image_length", type=int, default=50)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--iterations", type=int, default=30000)
    ap.add_argument("--densification_interval", type=int, default=100)
    ap.add_argument("--num_points", type=int, default=10000)
    ap.add_argument("--loss_type", type=str, default="L2")
    ap.add_argument("--seed", type=float, default=1)
    ap.add_argument("--removal_rate", type=float, default=0.1)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--is_ad", action="store_true")
    ap.add_argument("--is_rm", action="store_true")
    ap.add_argument("--k_frames", type=str, default="auto",
                    help="auto (K_frames.txt, else detect), forced (shard boundaries only), "
                         "or a comma list")
    ap.add_argument("--root", type=str, default="./checkpoints")
    ap.add_argument("--ranks_per_gpu", type=int, default=1,
                    help="ranks sharing one GPU (each trains its own GOPs on its own stream; "
                         "> 1 uses gloo for the metric collectives, RCCL takes one rank per GPU)")
    return ap.parse_args(argv)


def rank_device(local: int, ranks_per_gpu: int, use_cuda: bool):
    """(device, backend) of a rank: GPU local // ranks_per_gpu.  Frames and
    GOPs are independent, and one frame's training step is a latency chain
    that leaves most of the GPU idle, so several ranks per GPU overlap their
    steps; their only collectives are the metric aggregate and the K-frame
    detector's gathers, so gloo (host) serves them when ranks share a GPU."""
    rpg = max(1, int(ranks_per_gpu))
    if not use_cuda:
        return torch.device("cpu"), "gloo"
    return torch.device("cuda", local // rpg), ("nccl" if rpg == 1 else "gloo")


def main(argv=None):
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available()
    device, args.backend = rank_device(local, args.ranks_per_gpu, use_cuda)
    if use_cuda:
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    if args.seed is not None:
        np.random.seed(int(args.seed))

    if args.dataset:
        size = args.width * args.height * 3 // 2
        total = os.path.getsize(args.dataset) // size
        num_frames = min(args.image_length, total)

        def frame_fn(i, _cache={}):
            if i not in _cache:
                _cache.clear()
                fr, _ = load_yuv_frames(args.dataset, args.width, args.height, device, [i])
                _cache.update(fr)
            return _cache[i]
    else:
        num_frames = args.synthetic or args.image_length
        make = textured_video if getattr(args, "synthetic_kind", "smooth") == "textured" else synthetic_video
        gen = make(num_frames, args.height, args.width, int(args.seed), args.cut_every, device=device)

        def frame_fn(i):
            return gen(i).to(device)

    base = Path(args.root) / args.savdir / args.data_name
    kfile = base / "K_frames.txt"
    had_kfile = kfile.exists()
    if args.k_frames == "forced":
        k_frames, source = [1], "forced"
    elif args.k_frames not in ("auto",):
        k_frames, source = sorted({1} | {int(x) for x in args.k_frames.split(",") if x.strip()}), "list"
    elif had_kfile:  # the reference's cache (train_video_Represent.py:312-316)
        k_frames, source = [int(x) for x in kfile.read_text().split()], "file"
    else:
        k_frames, source = detect_k_frames(frame_fn, num_frames, rank, world, args.loss_type,
                                           args.lr, seed=int(args.seed)), "detected"
    # too few GOPs for the ranks: K-frames forced at equal-frame shard
    # boundaries
    if len(gops(k_frames, num_frames)) < world:
        k_frames = sorted(set(k_frames) | set(forced_k_frames(num_frames, world)))
    if rank == 0:
        base.mkdir(parents=True, exist_ok=True)
        # the GOPs this run trained; K_frames.txt (which the reference reads) is
        # written only when it did not exist and the list came from detection,
        # so a reference run on the same directory trains the same GOPs --
        # never overwritten
        (base / "K_frames_used.txt").write_text("".join(f"{k}\n" for k in k_frames))
        if not had_kfile and source == "detected":
            kfile.write_text("".join(f"{k}\n" for k in k_frames))

    t0 = time.time()
    res = train_video(frame_fn, num_frames, k_frames, args, rank, world, device)
    wall = time.time() - t0
    out_dir = base / f"{args.model_name}_{args.iterations}_{args.num_points}"
    out_dir.mkdir(parents=True, exist_ok=True)
    mdir = Path(args.root) / args.savdir_m / args.data_name / f"{args.model_name}_{args.iterations}_{args.num_points}"
    mdir.mkdir(parents=True, exist_ok=True)
    # one gmodels_state_dict.pth keyed frame_<n> (train_video_Represent.py:379,384):
    # rank 0 gathers every rank's frames
    models = res["models"]
    d = _dist()
    if d is not None:
        parts = [None] * world if rank == 0 else None
        d.gather_object(models, parts, dst=0)
        if rank == 0:
            models = {}
            for part in parts:
                models.update(part)
    if rank == 0:
        order = sorted(models, key=lambda k: int(k.split("_")[1]))
        torch.save({k: models[k] for k in order}, mdir / "gmodels_state_dict.pth")
    with open(out_dir / f"train_rank{rank}.jsonl", "w") as fh:
        for r in res["frames"]:
            fh.write(json.dumps(r) + "\n")
    if rank == 0:
        avg = res["average"]
        line = dict(frames=avg["frames"], ranks=world, wall_s=wall, k_frames=k_frames,
                    avg_psnr=avg["psnr"], avg_ms_ssim=avg["ms_ssim"],
                    avg_training_time=avg["training_time"], avg_eval_time=avg["eval_time"],
                    avg_eval_fps=avg["eval_fps"], avg_gaussians=avg["num_gaussians"])
        with open(out_dir / "train.txt", "a") as fh:
            fh.write(json.dumps(line) + "\n")
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
