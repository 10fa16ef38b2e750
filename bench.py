"""Benchmark of the GSVC hot path on MI355X (driver contract: one JSON line).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[1]): render one 1920x1080 frame of 10,000
splats, i.e. ``GaussianVideoFrame.forward()`` (the restatement of GSVC's
GaussianSplats_Represent.py:83-90: project -> bin/sort -> sum-rasterize ->
clamp -> NCHW), the loop train_video_Represent.py:103-106 times for its FPS.
A step is one frame.  Each rank renders its own synthetic frame (random-init
splats, seeded per rank): frames shard across GPUs with no data-path
collective (weak scaling); ranks only all-reduce their timings.

Reported beside the primary value:
  roofline      composite kernel (rasterize_sum_forward): algorithmic bytes per
                launch (36 N_vis + 4 M_eff + 8 T + 12 P) over its
                average duration from HIP events on its stream, vs 8 TB/s;
                ``traffic`` = PMC HBM bytes per launch from profiles/ (rocprofv3).
  cpu_baseline  the CPU oracle (oracle/oracle.c, single thread) rendering the
                same frame, timed on a bounded sample on this host.
  secondary     BASELINE configs[2]: 1080p / 50k splats full train_iter
                (L2 + backward + Adan) iterations/s and 50k render fps (N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402

METRIC = "1920×1080 frames/sec (render + train-iter) @ N splats; PSNR vs ref"
H, W = 1080, 1920
HBM_PEAK_GBS = 8000.0
PUBLISHED_FPS = 1500.0  # BASELINE.md §1 (README.md:19; splat count unstated)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--splats", type=int, default=10000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing", choices=["dispatch", "marker"], default="dispatch",
                    help="composite-kernel HIP events: carried by the timed dispatch "
                         "(hipExtLaunchKernel) or recorded around it")
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def all_max(x, world, device):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def composite_bytes_of(means2d, L, tile_bounds):
    """SURVEY §8d B_fwd = 36 N_vis + 4 M_eff + 8 T + 12 P for the render
    (inference) forward of one frame: the [3,H,W] clamped image is written
    once and no final_idx (the 16 P of the autograd forward counts its 4 B/px
    final_idx)."""
    from gsvc_amd import ops
    from gsvc_amd.utils import bin_and_sort_for_raster
    n = means2d.shape[0]
    with torch.no_grad():
        xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(
            n, means2d, L, H, W, tile_bounds, 0.01)
        m, gids, bins = bin_and_sort_for_raster(n, xys, depths, radii, nth, tile_bounds)
        if bins is None:
            m_eff = 0
        else:
            m_eff = int((bins[:, 1] - bins[:, 0]).clamp(min=0, max=256).sum())
        n_vis = int((nth > 0).sum())
    T = tile_bounds[0] * tile_bounds[1]
    P = H * W
    return 36 * n_vis + 4 * m_eff + 8 * T + 12 * P, dict(N_vis=n_vis, M=m, M_eff=m_eff, T=T, P=P)


def composite_bytes(model):
    return composite_bytes_of(model.get_xyz.detach(), model.get_cholesky_elements.detach(),
                              model.tile_bounds)


def load_profile(n_splats):
    """(PMC HBM bytes per launch, rocprofv3 kernel-trace average duration in
    us) of the composite kernel from profiles/pmc_traffic.json (written by
    tools/gpu_bench_prof.sh from rocprofv3 runs of this same command)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(str(n_splats), {})
        return (rec.get("rasterize_sum_forward_bytes_per_launch"),
                rec.get("rasterize_sum_forward_trace_avg_us"))
    except (OSError, ValueError):
        return None, None


def cpu_baseline(n_splats, seconds):
    """The CPU oracle rendering the workload's frame on this host: 1 thread
    (``value``) and every core this process may use (``all_cores``; the
    per-tile loop of the sum rasterizer in OpenMP, the binning serial)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    means, L, colors, opac = O.synthetic_frame(n_splats, seed=0)

    def rate(threads, budget):
        O.set_threads(threads)
        O.render_sum(means, L, colors, opac, H, W)  # warm-up / lib build
        t0 = time.perf_counter()
        frames = 0
        while True:
            O.render_sum(means, L, colors, opac, H, W)
            frames += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return frames, el

    # the box's CPU share: OMP_NUM_THREADS (16 per GPU there), at most the affinity set
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    f1, e1 = rate(1, seconds)
    fn, en = rate(cores, max(2.0, seconds / 3))
    O.set_threads(1)
    return {"value": f1 / e1, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{f1} renders of one 1920x1080 / {n_splats}-splat frame "
                      f"(project+bin+sort+sum-raster) by oracle/oracle.c, 1 thread, {e1:.1f} s",
            "all_cores": {"value": fn / en, "cores": cores,
                          "sample": f"{fn} renders, OpenMP per-tile rasterizer, {en:.1f} s"}}


def video_decode(device, frames=8, splats=10000, steps=50, warmup=5):
    """A GOP of ``frames`` distinct 1920x1080 frame models (10k splats each,
    the reference init distributions) rendered by ONE gsvc_render_frames_sum
    call per step -- a video decoder's workload; the composite kernel then
    spans frames x tiles.  Reported beside (not instead of) the single-frame
    headline."""
    from gsvc_amd import ops
    from gsvc_amd.render import render_frames_sum
    g = torch.Generator().manual_seed(4242)
    xyz = torch.atanh(2 * (torch.rand(frames * splats, 2, generator=g) - 0.5)).to(device)
    chol = torch.rand(frames * splats, 3, generator=g).to(device)
    feat = torch.rand(frames * splats, 3, generator=g).to(device)
    bound = torch.tensor([0.5, 0.0, 0.5], device=device)
    bg = torch.ones(3, device=device)
    sizes = [splats] * frames
    for _ in range(warmup):
        render_frames_sum(xyz, chol, feat, sizes, H, W, bg, cholesky_bound=bound)
    torch.cuda.synchronize()
    ops.composite_timing(True, max_launches=steps, every=4)
    t0 = time.perf_counter()
    for _ in range(steps):
        render_frames_sum(xyz, chol, feat, sizes, H, W, bg, cholesky_bound=bound)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kt = ops.composite_times_ms(steps)
    ops.composite_timing(False)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    nbytes = 0
    for b in range(frames):
        sl = slice(b * splats, (b + 1) * splats)
        nb, _ = composite_bytes_of(torch.tanh(xyz[sl]), chol[sl] + bound, tb)
        nbytes += nb
    avg_ms = sum(kt) / len(kt)
    ach = nbytes / (avg_ms * 1e-3) / 1e9
    return {"workload": f"GOP of {frames} distinct 1920x1080 frame models x {splats} splats, one "
                        "gsvc_render_frames_sum call per step",
            "frames_per_s": frames * steps / el, "ms_per_call": 1e3 * el / steps,
            "roofline": {"kernel": "rasterize_sum_forward (frames x tiles)", "bound": "hbm",
                         "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "avg_kernel_us": round(avg_ms * 1e3, 2),
                         "algorithmic_bytes_per_launch": nbytes}}


def secondary(device, steps=50, warmup=10):
    """configs[2]: 1080p / 50k splats train_iter and render (N=1 only)."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    model = make_frame_model(H, W, 50000, device, seed=7)
    gt = synthetic_gt(H, W, 8, device)
    for it in range(1, warmup + 1):
        model.train_iter(gt, it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    psnr = 0.0
    for it in range(warmup + 1, warmup + steps + 1):
        _, psnr = model.train_iter(gt, it)
    torch.cuda.synchronize()
    t_train = (time.perf_counter() - t0) / steps
    with torch.no_grad():
        for _ in range(warmup):
            model()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            model()
        torch.cuda.synchronize()
        t_render = (time.perf_counter() - t0) / steps
    return {"workload": "1920x1080, 50000 splats (BASELINE configs[2])",
            "train_iters_per_s": 1.0 / t_train, "train_ms_per_iter": 1e3 * t_train,
            "render_fps": 1.0 / t_render, "psnr_after_iters": psnr,
            "train_iter": "forward + L2 + backward + PSNR .item() + Adan + zero_grad + StepLR",
            "train_iter_path": ("fused: gsvc_train_step_sum (projection+slabs, per-tile "
                                "forward/loss/backward, per-splat VJP+Adan)"
                                if model.fused_steps else "op by op")}


def main():
    args = parse()
    world, rank, local = dist_setup()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    from gsvc_amd import ops
    from gsvc_amd.frame import make_frame_model

    model = make_frame_model(H, W, args.splats, device, seed=1000 + rank)
    model.eval()
    with torch.no_grad():
        for _ in range(args.warmup):
            model()
        torch.cuda.synchronize()
        # HIP events around every 16th composite launch of the timed region,
        # recorded by the library on the kernel's own stream
        ops.composite_timing(True, max_launches=args.steps, every=16,
                             dispatch=args.timing == "dispatch")
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            model()
        torch.cuda.synchronize()
        # each rank's clock stops at its own synchronize; the closing barrier
        # still brackets the region, and the max over ranks (all_max below) is
        # the job's time -- the barrier's own RCCL latency is not frame time
        elapsed = time.perf_counter() - t0
        barrier(world)
        kt = ops.composite_times_ms(args.steps)
        ops.composite_timing(False)
    elapsed = all_max(elapsed, world, device)
    value = world * args.steps / elapsed

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    nbytes, shape = composite_bytes(model)
    avg_ms = sum(kt) / len(kt)
    achieved = nbytes / (avg_ms * 1e-3) / 1e9
    traffic, trace_us = load_profile(args.splats)
    roof = {"kernel": "rasterize_sum_forward", "bound": "hbm", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "avg_kernel_us": round(avg_ms * 1e3, 2),
            "algorithmic_bytes_per_launch": nbytes, "shape": shape,
            "timing": ("HIP events carried by every 16th composite dispatch (hipExtLaunchKernel)"
                       if args.timing == "dispatch" else
                       "HIP events recorded around every 16th composite launch")}
    if trace_us:
        # the same kernel's duration in the committed rocprofv3 kernel trace
        # (marker events around the launch add ~3 us of packet / dispatch latency)
        roof["trace_avg_kernel_us"] = round(trace_us, 2)
        roof["frac_by_trace"] = round(nbytes / (trace_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": round(value / PUBLISHED_FPS, 3), "dtype": "f32",
        "data": "synthetic (random-init splats, reference init distributions)",
        "config": {"workload": f"render 1920x1080, {args.splats} splats (BASELINE configs[1]): "
                               "GaussianVideoFrame.forward = project + bin/sort + sum-raster + "
                               "clamp + NCHW", "H": H, "W": W, "splats": args.splats,
                   "parallelism": f"frames sharded over {world} rank(s), no data-path collective"},
        "roofline": roof,
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.splats, args.cpu_seconds)
    if world == 1 and not args.no_secondary:
        line["secondary"] = secondary(device)
        line["video_decode"] = video_decode(device)
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
