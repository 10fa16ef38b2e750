"""Benchmark of the GSVC hot path on MI355X (driver contract: one JSON line).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Headline workload (BASELINE.json configs[2], the configuration BASELINE.md §2
and ``north_star`` set the bar on): one ``GaussianVideoFrame.train_iter`` of a
1920x1080 frame with 50,000 splats -- the restatement of GSVC's
GaussianSplats_Represent.py:191-207 (forward = project -> bin -> sum-raster ->
clamp -> NCHW, L2 loss, backward, PSNR ``.item()``, Adan step, zero_grad,
StepLR), the loop train_video_Represent.py:85-96 runs per frame.  A step is one
training iteration; ``value`` is training iterations per second over all
ranks.  Each rank trains its own synthetic frame (random-init splats with the
reference's init distributions, seeded per rank; a seeded procedural target):
frames shard across GPUs with no data-path collective (weak scaling); ranks
only all-reduce their timings.

``python bench.py --gpus N`` with no torch.distributed environment starts N
rank processes itself (``torch.distributed.run`` as a child process; this
process never touches the GPU) and exits with their status.

Reported beside the primary value:
  roofline      the dominant kernel of the step (train_tile_band_kernel): algorithmic
                bytes per launch (12 P + 36 N_vis + 4 M_eff + 8 T +
                36 N) over its average duration from HIP events carried by its
                own dispatches (on its stream), vs 8 TB/s; ``traffic`` = PMC HBM
                bytes per launch from the committed rocprofv3 passes (profiles/),
                ``traffic_model`` = the bytes the slab design moves.
  kernels       every kernel of the step, event-timed the same way.
  render        configs[2]'s render: GaussianVideoFrame.forward at 50k splats,
                frames/s and the composite kernel's roofline.
  psnr_vs_ref   the fused trajectory against the reference's own train_iter run
                on CPU (tests/golden/train_traj_1080p_n50k.npz, make_golden.py).
  cpu_baseline  the CPU restatement (oracle/oracle.py train_iter_sum, C kernels)
                on the same settled state, k = 1 and all cores, median of 5.
  render_10k    configs[1] (render only, 10k splats) and ``video_decode``.
  op_path       the unchanged-caller path (GSVC's own files over the gsplat
                drop-in: autograd op by op): forward, forward + backward, render
                fps and train-iters/s at the same trained frame, with the
                composite's and the backward kernel's rooflines.
  alpha         the alpha-compositing operators (rasterize_gaussians) at
                1080p / 50k: forward, forward + backward, kernel rooflines.
  config0_cpu   BASELINE configs[0] (256x256, 1k splats) on the CPU.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402

METRIC = "1920×1080 frames/sec (render + train-iter) @ N splats; PSNR vs ref"
H, W = 1080, 1920
HBM_PEAK_GBS = 8000.0
TRAJ_FIXTURE = os.path.join(REPO, "tests", "golden", "train_traj_1080p_n50k.npz")
STATE_FIXTURE = os.path.join(REPO, "tests", "golden", "train_state_1080p_n50k.npz")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--settle", type=int, default=2000,
                    help="training iterations before the warmup (untimed): the timed steps "
                         "run at a trained splat density, not at random init")
    ap.add_argument("--timing-launches", type=int, default=200,
                    help="launches per kernel timed by HIP events after the timed region")
    ap.add_argument("--deterministic", action="store_true",
                    help="torch.use_deterministic_algorithms(True): the bitwise reproducible backward")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--knob", action="append", default=[],
                    help="A/B knob K=V (gsvc_debug_set) for kernel-variant comparisons")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: start the ranks, all-reduce, print the line (tests)")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """--gpus N without a torch.distributed environment: run N ranks of this
    script under torch.distributed.run in a child process (one process per
    GPU).  This process does not initialise the GPU and does not exec."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("GSVC_BENCH_SHARED_GPU") == "1" and args.backend != "nccl":
        local = 0  # rehearsal of N ranks on a one-GPU box (gloo): all ranks on cuda:0
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        import torch.distributed as dist
        if args.dry_run or args.backend != "nccl":
            dist.init_process_group(args.backend)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # every rank present: one all-reduce of ones
        dev = torch.device("cpu") if args.dry_run or args.backend != "nccl" else torch.device("cuda", local)
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        if int(t.item()) != world:
            raise SystemExit(f"bench.py: all-reduce saw {int(t.item())} ranks, expected {world}")
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


def frame_shape(means2d, L, tile_bounds):
    """N_vis, M and M_eff = sum over tiles of min(count, 256) of one frame (the
    op path's binning of the same splats), for the algorithmic byte counts."""
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
    return dict(N_vis=n_vis, M=int(m), M_eff=m_eff, T=tile_bounds[0] * tile_bounds[1], P=H * W)


def composite_bytes(shape):
    """SURVEY §8d B_fwd for the render (inference) forward: 36 N_vis + 4 M_eff +
    8 T + 12 P (the [3,H,W] clamped image written once, no final_idx)."""
    return 36 * shape["N_vis"] + 4 * shape["M_eff"] + 8 * shape["T"] + 12 * shape["P"]


def op_composite_bytes(shape):
    """The op path's autograd forward: the render's bytes (the image in HWC,
    12 P) plus the tiles' sorted ids and bins written back for the backward
    (4 M_eff + 8 T).  No final_idx: the round-5 backward does not read it
    (SURVEY §8d's B_fwd counts the reference's 4 P of it)."""
    return composite_bytes(shape) + 4 * shape["M_eff"] + 8 * shape["T"]


def sum_bwd_bytes(shape, n):
    """SURVEY §8d B_bwd without final_idx (the round-5 kernel does not read it):
    v_out 12 P + the visible splats 36 N_vis + the tile id lists 4 M_eff + bins
    8 T (read) + the gradients 36 N (written)."""
    return 12 * shape["P"] + 36 * shape["N_vis"] + 4 * shape["M_eff"] + 8 * shape["T"] + 36 * n


def alpha_fwd_bytes(shape):
    """The alpha forward (forward.cu:252-374): the visible splats 36 N_vis, every
    entry of the tile lists 4 M (no 256 cap) and bins 8 T (read); out 12 P,
    final_Ts 4 P, final_idx 4 P (written)."""
    return 36 * shape["N_vis"] + 4 * shape["M"] + 8 * shape["T"] + 20 * shape["P"]


def alpha_bwd_bytes(shape, n):
    """The alpha backward (backward.cu:138-315): v_out 12 P, v_out_alpha 4 P,
    final_Ts 4 P, final_idx 4 P, 36 N_vis + 4 M + 8 T (read); the gradients
    36 N (written)."""
    return 24 * shape["P"] + 36 * shape["N_vis"] + 4 * shape["M"] + 8 * shape["T"] + 36 * n


def train_tile_bytes(shape, n):
    """Algorithmic HBM bytes of one fused training tile pass (forward + loss +
    backward over every tile): the target frame 12 P, the
    visible splats' geometry and colour 36 N_vis, the tile id lists 4 M_eff and
    bins 8 T (read); the gradients 36 N (9 floats per splat, written).  The
    image, final_idx and v_out never leave the chip."""
    return 12 * shape["P"] + 36 * shape["N_vis"] + 4 * shape["M_eff"] + 8 * shape["T"] + 36 * n


def train_tile_traffic_model(shape):
    """What train_tile_band_kernel's design moves per launch:
    gt 12 P + tile counts 4 T + the tiles' 48-byte slab records 48 M_eff (read);
    gradient sums by atomics 32 M_eff (8 floats per (splat, tile)) + per-tile
    error sums 8 T + the next frame's count reset 4 T (written).  Reported next
    to the PMC traffic; the excess over train_tile_bytes is the slab design's."""
    return 12 * shape["P"] + 4 * shape["T"] + 48 * shape["M_eff"] + 32 * shape["M_eff"] + 12 * shape["T"]


def project_bytes(shape, n):
    """frame_project_kernel in the training step: parameters 36 N (xyz, chol,
    features, rgb_W) read; record 48 N + xys/radii 12 N + zeroed gradient
    record 64 N + the tiles' records 48 M + slot counters 4 M (write)."""
    return 36 * n + 48 * n + 12 * n + 64 * n + 52 * shape["M"]


def train_splat_bytes(n):
    """train_splat_kernel: gradient record 64 N + record 32 N + radii 4 N +
    parameters and Adan state (8 elements x (4 + 16 B)) read, parameters and
    state (8 x 20 B) written per splat; the 8 T loss sum is not counted."""
    return n * (64 + 32 + 4 + 8 * 20 + 8 * 20)


def load_profile(key):
    """PMC HBM bytes and kernel-trace durations per launch from
    profiles/pmc_traffic.json (tools/prof_summary.py over the committed
    rocprofv3 runs of this command)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(key, {})
    except (OSError, ValueError):
        return {}


def _avg(xs):
    return sum(xs) / len(xs) if xs else float("nan")


def roofline(kernel, nbytes, times_ms, prof=None, prof_key=None, timing=None):
    avg_ms = _avg(times_ms)
    achieved = nbytes / (avg_ms * 1e-3) / 1e9
    r = {"kernel": kernel, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
         "traffic": None, "avg_kernel_us": round(avg_ms * 1e3, 2),
         "timed_launches": len(times_ms),
         "algorithmic_bytes_per_launch": nbytes,
         "timing": timing or "HIP events carried by the kernel's own dispatches (hipExtLaunchKernel)"}
    if prof and prof_key:
        r["traffic"] = prof.get(f"{prof_key}_bytes_per_launch")
        tus = prof.get(f"{prof_key}_trace_avg_us")
        if tus:
            r["trace_avg_kernel_us"] = round(tus, 2)
            r["frac_by_trace"] = round(nbytes / (tus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    return r


VALU_PEAK_GINST = 256 * 4 * 2.4 / 2  # G wave64 VALU instructions/s (2 cycles each per SIMD)


def valu_roofline(kernel_key, avg_us):
    """The compute-side bound of a tile kernel: its PMC VALU wave-instructions
    per launch (profiles/pmc_valu.json, committed rocprofv3 pass) over the
    measured launch time, against the chip's VALU issue rate."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_valu.json")) as f:
            d = json.load(f)[kernel_key]
    except (OSError, ValueError, KeyError):
        return None
    insts = d["SQ_INSTS_VALU"]
    achieved = insts / (avg_us * 1e-6) / 1e9
    return {"bound": "valu", "insts_per_launch": insts, "achieved": round(achieved, 1),
            "peak": VALU_PEAK_GINST, "unit": "G wave-instructions/s",
            "frac": round(achieved / VALU_PEAK_GINST, 4), "source": "profiles/pmc_valu.json"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(n_splats, reps=5, warm=2):
    """The CPU restatement of the same training iteration (oracle/oracle.py
    train_iter_sum: project + bin + sum-raster + clamp + L2 + raster and
    projection VJPs + Adan; C kernels, OpenMP over tiles, numpy glue) on the
    SETTLED state the GPU is timed on (tests/golden/train_state_1080p_n50k.npz,
    the bench's frame after settle + warmup iterations), BASELINE.md §4
    protocol: k = 1 and k = all cores of this process's affinity, median of
    ``reps`` iterations after ``warm`` warm-ups each (all cores = the affinity
    mask, capped by OMP_NUM_THREADS: the GPU box grants 16 CPUs per GPU while
    its affinity mask shows the whole machine)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from gsvc_amd.frame import synthetic_gt
    if not os.path.exists(STATE_FIXTURE):
        return None
    z = np.load(STATE_FIXTURE)
    if n_splats != int(z["n"]):
        return None
    gt = synthetic_gt(H, W, int(z["gt_seed"]), "cpu").numpy()[0]
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():  # the box's CPU share (16 per GPU)
        cores = min(cores, max(1, int(os.environ["OMP_NUM_THREADS"])))
    runs = {}
    for k in sorted({1, cores}):
        O.set_threads(k)
        params = {name: np.array(z["state_" + name], copy=True)
                  for name in ("_xyz", "_cholesky", "_features_dc")}
        state = {}
        ts = []
        for i in range(warm + reps):
            t0 = time.perf_counter()
            O.train_iter_sum(params, gt, H, W, state, i + 1)  # Adan's own step count
            ts.append(time.perf_counter() - t0)
        ts = sorted(ts[warm:])
        runs[k] = ts[len(ts) // 2]
    O.set_threads(1)
    best = min(runs, key=runs.get)
    return {"value": 1.0 / runs[best], "unit": "train-iters/s", "cores": best, "kind": "port",
            "cpu_model": _cpu_model(),
            "per_cores": {str(k): round(1.0 / v, 4) for k, v in runs.items()},
            "sample": f"median of {reps} train iterations after {warm} warm-ups, per core count, "
                      f"of one 1920x1080 / {n_splats}-splat frame at the settled state the GPU "
                      f"times (after {int(z['iters'])} iterations, M = {int(z['M'])}; "
                      "oracle/oracle.py train_iter_sum: C project/bin/raster + VJPs with OpenMP "
                      "over tiles, numpy clamp/L2/Adan)"}


def _cpu_cores():
    """This process's CPU share: the affinity mask, capped by OMP_NUM_THREADS
    (the GPU box grants 16 CPUs per GPU while its mask shows the machine)."""
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, max(1, int(os.environ["OMP_NUM_THREADS"])))
    return cores


def _median_s(fn, reps, warm):
    ts = []
    for _ in range(warm + reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[warm:])
    return ts[len(ts) // 2]


def cpu_render_baseline(means, L, colors, H_, W_, label, reps=5, warm=2, backward=False):
    """The CPU baselines of one frame render (BASELINE.md §4 protocol, SURVEY
    §8d; the FPS loop of train_video_Represent.py:101-106): the oracle
    restatement (oracle/oracle.py render_sum: C project / bin / sum-raster,
    numpy glue; kind "port") and this package's own CPU dispatch of the two
    operators (gsplat.project_gaussians_2d + rasterize_gaussians_sum on CPU
    tensors, libgsvc_amd_cpu.so: the reference's "PyTorch-CPU fallback"
    config), each at k = 1 and k = all cores, median of ``reps`` frames after
    ``warm`` warm-ups.  Inputs: activated means2d [N,2], L [N,3], colours
    [N,3] (CPU float32).  ``backward``: also forward + backward of the CPU
    dispatch (v_out = ones)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from gsvc_amd import cpu as C
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    n = means.shape[0]
    mn, Ln, cn = (np.ascontiguousarray(t.numpy(), dtype=np.float32) for t in (means, L, colors))
    on = np.ones((n, 1), np.float32)
    tb = ((W_ + 15) // 16, (H_ + 15) // 16, 1)
    ones = torch.ones(n, 1)
    bg = torch.ones(3)

    def product_fwd():
        xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H_, W_, tb)
        rasterize_gaussians_sum(xys, depths, radii, conics, nth, colors, ones, H_, W_, 16, 16,
                                background=bg)

    def product_fwd_bwd():
        m, l, c = (t.clone().requires_grad_(True) for t in (means, L, colors))
        xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H_, W_, tb)
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, ones, H_, W_, 16, 16,
                                      background=bg)
        out.sum().backward()

    cores = _cpu_cores()
    per = {"oracle": {}, "product_cpu": {}}
    if backward:
        per["product_cpu_fwd_bwd"] = {}
    torch_threads = torch.get_num_threads()
    for k in sorted({1, cores}):
        O.set_threads(k)
        C.set_threads(k)
        torch.set_num_threads(k)
        per["oracle"][str(k)] = round(1.0 / _median_s(lambda: O.render_sum(mn, Ln, cn, on, H_, W_),
                                                      reps, warm), 3)
        with torch.no_grad():
            per["product_cpu"][str(k)] = round(1.0 / _median_s(product_fwd, reps, warm), 3)
        if backward:
            per["product_cpu_fwd_bwd"][str(k)] = round(1.0 / _median_s(product_fwd_bwd, reps, warm), 3)
    O.set_threads(1)
    C.set_threads(cores)
    torch.set_num_threads(torch_threads)
    best_k = max(per["oracle"], key=per["oracle"].get)
    return {"value": per["oracle"][best_k], "unit": "frames/s", "cores": int(best_k), "kind": "port",
            "cpu_model": _cpu_model(), "per_path_per_cores": per,
            "sample": f"median of {reps} renders after {warm} warm-ups per path and core count, "
                      f"{label}: {W_}x{H_}, {n} splats; value = the oracle restatement "
                      "(oracle/oracle.py render_sum: C project/bin/sum-raster, numpy glue); "
                      "product_cpu = gsplat ops on CPU tensors (libgsvc_amd_cpu.so, OpenMP)"}


def config0_cpu(reps=5, warm=2):
    """BASELINE configs[0]: a single 256x256 synthetic frame, 1k splats, on the
    CPU (the reference's PyTorch-CPU rasterize case): forward and forward +
    backward through the operators' CPU dispatch, and the oracle."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    means, L, colors, _ = O.synthetic_frame(1000, 0)
    r = cpu_render_baseline(torch.from_numpy(np.ascontiguousarray(means, np.float32)),
                            torch.from_numpy(np.ascontiguousarray(L, np.float32)),
                            torch.from_numpy(np.ascontiguousarray(colors, np.float32)),
                            256, 256, "BASELINE configs[0] (synthetic frame, seed 0)", reps, warm,
                            backward=True)
    r["workload"] = "BASELINE configs[0]: one 256x256 frame, 1k splats, CPU only"
    return r


def psnr_vs_ref(device):
    """Run the reference trajectory's iterations (same seed, init, target) on
    the fused path and compare per-iteration PSNR with the reference's CPU run."""
    import numpy as np
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    z = np.load(TRAJ_FIXTURE)
    n, iters = int(z["n"]), int(z["iters"])
    model = make_frame_model(int(z["H"]), int(z["W"]), n, device, seed=int(z["seed"]))
    gt = synthetic_gt(int(z["H"]), int(z["W"]), int(z["gt_seed"]), "cpu").to(device)
    ps = []
    for it in range(1, iters + 1):
        _, p = model.train_iter(gt, it)
        ps.append(p)
    ref = [float(x) for x in z["psnrs"]]
    d = [abs(a - b) for a, b in zip(ps, ref)]
    return {"iters": iters, "psnr": round(ps[-1], 6), "psnr_ref": round(ref[-1], 6),
            "max_abs_diff_db": float(f"{max(d):.3g}"),
            "fused_steps": model.fused_steps,
            "ref": "GaussianVideo_frame.train_iter (reference Python, oracle kernels, CPU), "
                   "tests/golden/train_traj_1080p_n50k.npz"}


def time_channels(channels, fn, launches):
    """HIP-event durations (ms) of every launch of ``channels`` while calling
    ``fn`` ``launches`` times (outside the timed region)."""
    from gsvc_amd import ops
    for c in channels:
        ops.channel_timing(c, True, max_launches=launches, every=1, dispatch=True)
    for _ in range(launches):
        fn()
    torch.cuda.synchronize()
    out = {c: ops.channel_times_ms(c, launches) for c in channels}
    for c in channels:
        ops.channel_timing(c, False)
    return out


def render_block(model, steps, warmup):
    """configs[2]'s render: GaussianVideoFrame.forward() of the trained model."""
    from gsvc_amd import ops
    with torch.no_grad():
        for _ in range(warmup):
            model()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            model()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        times = time_channels(["composite", "project"], model, 200)
    shape = frame_shape(model.get_xyz.detach(), model.get_cholesky_elements.detach(),
                        model.tile_bounds)
    prof = load_profile(f"render_{model._xyz.shape[0]}")
    roof = roofline("raster_render_ids_kernel (composite: the single-frame render)", composite_bytes(shape),
                    times["composite"], prof, "rasterize_sum_forward")
    vr = valu_roofline(f"render_{model._xyz.shape[0]}",
                       roof.get("trace_avg_kernel_us") or roof["avg_kernel_us"])
    if vr:
        roof["valu"] = vr
    return {"workload": f"GaussianVideoFrame.forward, 1920x1080, {model._xyz.shape[0]} splats "
                        "(configs[2] render): project + bin + sum-raster + clamp + NCHW",
            "frames_per_s": round(steps / el, 1), "ms_per_frame": round(1e3 * el / steps, 4),
            "roofline": roof,
            "project_avg_us": round(_avg(times["project"]) * 1e3, 2), "shape": shape}


def render10k_model(device):
    from gsvc_amd.frame import make_frame_model
    model = make_frame_model(H, W, 10000, device, seed=1000)
    model.eval()
    return model


def render_10k(device, steps=200, warmup=20):
    """configs[1]: render one 1920x1080 frame of 10k splats."""
    model = render10k_model(device)
    r = render_block(model, steps, warmup)
    r["workload"] = r["workload"].replace("(configs[2] render)", "(configs[1])")
    return r


def video_decode(device, frames=8, splats=10000, steps=50, warmup=5):
    """A GOP of ``frames`` distinct 1920x1080 frame models (10k splats each)
    rendered by ONE gsvc_render_frames_sum call per step (a decoder's workload)."""
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
    ops.composite_timing(True, max_launches=steps, every=1, dispatch=True)
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
        nbytes += composite_bytes(frame_shape(torch.tanh(xyz[sl]), chol[sl] + bound, tb))
    return {"workload": f"GOP of {frames} distinct 1920x1080 frame models x {splats} splats, one "
                        "gsvc_render_frames_sum call per step",
            "frames_per_s": round(frames * steps / el, 1), "ms_per_call": round(1e3 * el / steps, 4),
            "roofline": roofline("raster_sum_fwd_kernel (frames x tiles)", nbytes, kt,
                                 load_profile("video_decode"), "rasterize_sum_forward")}


def op_path_block(model, gt, device, steps=200, warmup=20):
    """The unchanged-caller path: what GSVC's own
    GaussianSplats_Represent.py runs on the drop-in package -- autograd through
    gsplat.project_gaussians_2d / rasterize_gaussians_sum, then clamp + NCHW,
    L2, backward, PSNR .item(), the optimizer step (:83-90, :191-207) -- and its
    FPS loop's forward (train_video_Represent.py:101-106), on a copy of the
    bench's trained frame (fresh optimizer state, as a P-frame starts).
    ``train_iters_per_s`` uses gsvc_amd.adan.Adan (one fused update kernel);
    ``train_iters_per_s_foreach_adan`` the reference optimizer's own foreach
    sequence (tools/foreach_adan.py, op for op optimizer.py:296-362), i.e.
    GSVC's files with nothing changed but the gsplat package."""
    import math
    import torch.nn.functional as F
    from gsvc_amd.frame import make_frame_model
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from foreach_adan import ForeachAdan
    n = model._xyz.shape[0]
    op = make_frame_model(H, W, n, device, seed=0, fused_train=False, fused_render=False)
    with torch.no_grad():
        for k in ("_xyz", "_cholesky", "_features_dc"):
            getattr(op, k).copy_(getattr(model, k))
    assert not op.fused_train and not op.fused_render

    def timed(fn, k, w):
        # w calls and at least 0.3 s of them, then the median of three blocks
        # of k: right after the model's setup the host side ran slow for ~0.5 s
        # (forward + backward 310-330 us, then 180-200, tools/planar_ab.py,
        # profiles/r06/planar_op/), and one box's first forward block read
        # 159.8 us against 72.6 on the next (profiles/r06/final)
        t_w = time.perf_counter()
        for j in range(10 ** 7):
            fn()
            if j + 1 >= w and time.perf_counter() - t_w > 0.3:
                break
        blocks = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                fn()
            torch.cuda.synchronize()
            blocks.append((time.perf_counter() - t0) / k)
        return sorted(blocks)[1]

    def fwd():
        op.forward()

    def fwd_bwd():
        for p in (op._xyz, op._cholesky, op._features_dc):
            p.grad = None
        img = op.forward()["render"]
        F.mse_loss(img.squeeze(0), gt.squeeze(0)).backward()

    def render():
        with torch.no_grad():
            op.forward()

    it = [0]

    def train():
        it[0] += 1
        op.train_iter(gt, it[0])

    fopt = ForeachAdan([op._xyz, op._cholesky, op._features_dc], lr=op.lr)

    def train_foreach():  # GaussianSplats_Represent.py:191-207 with optimizer.py's Adan
        img = op.forward()["render"]
        loss = F.mse_loss(img.squeeze(0), gt.squeeze(0))
        loss.backward()
        with torch.no_grad():
            math.log10(1.0 / F.mse_loss(img, gt).item())
        fopt.step()
        for p in fopt.params:
            p.grad = None

    t_fwd = timed(fwd, steps, warmup)
    t_fb = timed(fwd_bwd, steps, warmup)
    t_render = timed(render, steps, warmup)
    t_train = timed(train, steps, warmup)
    t_train_fe = timed(train_foreach, steps, warmup)
    assert op.fused_steps == 0
    # the drop-in's own kernels in forward + backward calls, HIP events on
    # their dispatches (outside the timed loops)
    kt = time_channels(["composite", "sum_bwd"], fwd_bwd, 100)
    host = op_host_us(op, steps)
    shape = frame_shape(op.get_xyz.detach(), op.get_cholesky_elements.detach(), op.tile_bounds)
    prof = load_profile("op_path")
    return {"workload": f"unchanged-caller op path at 1920x1080 / {n} splats (the bench's trained "
                        "frame): autograd through gsplat.* + clamp + NCHW",
            "fwd_us": round(t_fwd * 1e6, 1), "fwd_bwd_us": round(t_fb * 1e6, 1),
            "render_fps": round(1.0 / t_render, 1),
            "train_iters_per_s": round(1.0 / t_train, 1),
            "train_iters_per_s_foreach_adan": round(1.0 / t_train_fe, 1),
            "timing": f"wall clock, median of 3 blocks of {steps} calls after >= {warmup} "
                      "warm-up calls and >= 0.3 s, synchronized",
            "host_us_per_call": host,
            "kernels": {
                "raster_sum_fwd": roofline("raster_sum_fwd_kernel (op path: id slabs, sorted-id write-back)",
                                           op_composite_bytes(shape), kt["composite"], prof,
                                           "rasterize_sum_forward"),
                "raster_sum_bwd": roofline("raster_sum_bwd_kernel", sum_bwd_bytes(shape, n),
                                           kt["sum_bwd"], prof, "rasterize_sum_backward")}}


def op_host_us(op, calls):
    """Host (CPU) time per call of the drop-in's own two operators on the
    frame's activations -- the C++ Functions' forward calls and their backward
    nodes, each call timed alone with the GPU work left asynchronous -- beside
    GSVC's own op sequence around them (the rest of op_path's wall time)."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    m = op.get_xyz.detach().clone().requires_grad_(True)
    L = op.get_cholesky_elements.detach().clone().requires_grad_(True)
    c = op.get_features.detach().clone().requires_grad_(True)
    o = torch.ones(m.shape[0], 1, device=m.device)
    bg = torch.ones(3, device=m.device)
    tb = op.tile_bounds
    v = torch.ones(H, W, 3, device=m.device)
    t = {"project_gaussians_2d": 0.0, "rasterize_gaussians_sum": 0.0, "backward_both": 0.0}
    for k in range(calls + 10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        xys, depths, radii, conics, nth = project_gaussians_2d(m, L, H, W, tb)
        t1 = time.perf_counter()
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                      background=bg)
        t2 = time.perf_counter()
        torch.autograd.grad(out, (m, L, c), v)
        t3 = time.perf_counter()
        if k >= 10:
            t["project_gaussians_2d"] += t1 - t0
            t["rasterize_gaussians_sum"] += t2 - t1
            t["backward_both"] += t3 - t2
    torch.cuda.synchronize()
    return {k: round(x / calls * 1e6, 1) for k, x in t.items()}


def alpha_block(device, n=50000, steps=100, warmup=10):
    """The alpha-compositing path north_star names (rasterize.py:14-253,
    forward.cu:252-374, backward.cu:138-315) through the drop-in operators at
    1920x1080: random-init splats with opacity U(0.1, 1) (tools/alphabench.py's
    workload), project_gaussians_2d + rasterize_gaussians per call, forward and
    forward + backward; each kernel's roofline from HIP events on its own
    dispatches."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize import rasterize_gaussians
    g = torch.Generator().manual_seed(n)
    means = torch.tanh(torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5))).to(device)
    L = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0, 0.5])).to(device)
    col = torch.rand(n, 3, generator=g).to(device)
    opac = (0.1 + 0.9 * torch.rand(n, 1, generator=g)).to(device)
    bg = torch.ones(3, device=device)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    params = [t.clone().requires_grad_(True) for t in (means, L, col, opac)]

    def fwd():
        with torch.no_grad():
            xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
            rasterize_gaussians(xys, depths, radii, conics, nth, col, opac, H, W, 16, 16, background=bg)

    def fwd_bwd():
        m, l, c, o = params
        xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
        out = rasterize_gaussians(xys, depths, radii, conics, nth, c, o, H, W, 16, 16, background=bg)
        torch.autograd.grad(out.sum(), params)

    def timed(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    t_f = timed(fwd)
    t_fb = timed(fwd_bwd)
    kt = time_channels(["alpha_fwd", "alpha_bwd"], fwd_bwd, 100)
    shape = frame_shape(means, L, tb)
    prof = load_profile("alpha_50000")
    return {"workload": f"rasterize_gaussians (alpha compositing) at 1920x1080 / {n} splats, random "
                        "init, opacity U(0.1, 1): project_gaussians_2d + rasterize_gaussians per call",
            "fwd_us": round(t_f * 1e6, 1), "fwd_bwd_us": round(t_fb * 1e6, 1),
            "kernels": {
                "raster_alpha_fwd": roofline("raster_alpha_fwd_kernel", alpha_fwd_bytes(shape),
                                             kt["alpha_fwd"], prof, "alpha_forward"),
                "raster_alpha_bwd": roofline("raster_alpha_bwd_kernel", alpha_bwd_bytes(shape, n),
                                             kt["alpha_bwd"], prof, "alpha_backward")},
            "shape": shape}


def dry_run(args, world, rank):
    """--dry-run: the rank plumbing without a GPU (tests/test_bench_launch.py)."""
    t0 = time.perf_counter()
    x = torch.ones(1000)
    for _ in range(args.steps):
        x = x * 1.0001
    elapsed = all_max(time.perf_counter() - t0, world, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(world * args.steps / elapsed, 2),
                          "unit": "train-iters/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "ranks_seen": world}), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world, rank, local = dist_setup(args)
    if args.dry_run:
        dry_run(args, world, rank)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    if args.knob:
        # A/B knobs exist only in the diagnostic library (an A/B run, not the headline)
        os.environ["GSVC_DIAG"] = "1"
        from gsvc_amd import _lib
        for kv in args.knob:
            k, v = kv.split("=")
            if _lib.load().gsvc_debug_set(int(k), int(v)) < 0:
                raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")

    if args.deterministic:
        torch.use_deterministic_algorithms(True, warn_only=True)
    # ---- headline: configs[2] training iterations, one frame per rank
    model = make_frame_model(H, W, args.splats, device, seed=1000 + rank)
    gt = synthetic_gt(H, W, 8 + rank, "cpu").to(device)
    it = 0
    psnr = float("nan")
    for _ in range(args.settle + args.warmup):
        it += 1
        model.train_iter(gt, it)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        it += 1
        _, psnr = model.train_iter(gt, it)
    torch.cuda.synchronize()
    # each rank's clock stops at its own synchronize; the closing barrier still
    # brackets the region and the max over ranks (all_max) is the job's time
    elapsed = time.perf_counter() - t0
    barrier(world)
    elapsed = all_max(elapsed, world, device)
    value = world * args.steps / elapsed

    # ---- per-kernel HIP-event timing of the step, outside the timed region
    state = {"it": it}

    def one_iter():
        state["it"] += 1
        model.train_iter(gt, state["it"])

    kt = time_channels(["train_tile", "project", "train_splat"], one_iter, args.timing_launches)
    shape = frame_shape(model.get_xyz.detach(), model.get_cholesky_elements.detach(),
                        model.tile_bounds)
    # N > 1: the render half of the metric, weak-scaled like the headline (each
    # rank renders its own trained frame; barrier-bracketed, max over ranks)
    render_ranks = None
    if world > 1 and not args.no_secondary:
        model.eval()
        with torch.no_grad():
            for _ in range(20):
                model()
            barrier(world)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(200):
                model()
            torch.cuda.synchronize()
            rel = time.perf_counter() - t1
        barrier(world)
        rel = all_max(rel, world, device)
        render_ranks = {"workload": "GaussianVideoFrame.forward of each rank's trained 1920x1080 "
                                    f"frame, {args.splats} splats, 200 frames per rank",
                        "frames_per_s": round(world * 200 / rel, 1),
                        "ms_per_frame": round(1e3 * rel / 200, 4), "ranks": world}
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    prof = load_profile(f"train_{args.splats}")
    roof = roofline("train_tile_band_kernel", train_tile_bytes(shape, args.splats), kt["train_tile"],
                    prof, "train_tile")
    roof["traffic_model"] = train_tile_traffic_model(shape)
    if roof.get("traffic"):
        roof["traffic_over_algorithmic"] = round(roof["traffic"] / roof["algorithmic_bytes_per_launch"], 3)
    # the tile kernel is VALU/latency bound at trained density:
    # its VALU issue fraction beside the HBM roofline
    vr = valu_roofline("train_tile", roof.get("trace_avg_kernel_us") or roof["avg_kernel_us"])
    if vr:
        roof["valu"] = vr
    kernels = {
        "train_tile": roof,
        "frame_project": roofline("frame_project_ordered_kernel", project_bytes(shape, args.splats),
                                  kt["project"], prof, "frame_project_ordered"),
        "train_splat": roofline("train_splat_kernel", train_splat_bytes(args.splats),
                                kt["train_splat"], prof, "train_splat"),
    }
    # GSVC_BENCH_SHARED_GPU (a rehearsal of N ranks on one GPU): the devices
    # used, not the ranks, are the GPU count
    shared = os.environ.get("GSVC_BENCH_SHARED_GPU") == "1" and args.backend != "nccl"
    n_gpus = 1 if shared else world
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "train-iters/s", "n_gpus": n_gpus,
        "steps": args.steps, "warmup": args.warmup, "settle_iters": args.settle,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (random-init splats with the reference init distributions, seeded "
                "procedural 1920x1080 target); the timed steps start after settle + warmup "
                "training iterations (trained splat density, ~2x the entries of random init)",
        "config": {"workload": f"BASELINE configs[2]: train_iter of one 1920x1080 frame, "
                               f"{args.splats} splats (GaussianVideoFrame.train_iter = forward + "
                               "L2 + backward + PSNR .item() + Adan + zero_grad + StepLR)",
                   "H": H, "W": W, "splats": args.splats,
                   "deterministic_backward": bool(args.deterministic),
                   "parallelism": f"one frame per rank, {world} rank(s), no data-path collective"
                                  + (f", all ranks sharing one GPU" if shared else "")},
        "ranks_per_gpu": world if shared else 1,
        "roofline": roof,
        "kernels": kernels,
        "shape": shape,
        "psnr_after_iters": round(psnr, 6),
        "train_iter_path": ("fused: gsvc_train_step_sum" if model.fused_steps else "op by op"),
        "cpu_baseline": None,
    }
    if render_ranks is not None:
        line["render"] = render_ranks
    if world == 1 and not args.no_secondary:
        line["psnr_vs_ref"] = psnr_vs_ref(device)
        model.eval()
        line["render"] = render_block(model, 200, 20)
        line["render"]["vs_published_1500fps"] = round(line["render"]["frames_per_s"] / 1500.0, 2)
        line["render_10k"] = render_10k(device)
        line["video_decode"] = video_decode(device)
        line["op_path"] = op_path_block(model, gt, device)
        line["alpha"] = alpha_block(device)
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.splats)
        if "render" in line:  # configs[2] render and configs[1]: the same frames on the CPU
            with torch.no_grad():
                line["render"]["cpu_baseline"] = cpu_render_baseline(
                    model.get_xyz.detach().cpu(), model.get_cholesky_elements.detach().cpu(),
                    model.get_features.detach().cpu().contiguous(), H, W,
                    "the bench's trained configs[2] frame")
                m10 = render10k_model(device)
                line["render_10k"]["cpu_baseline"] = cpu_render_baseline(
                    m10.get_xyz.detach().cpu(), m10.get_cholesky_elements.detach().cpu(),
                    m10.get_features.detach().cpu().contiguous(), H, W,
                    "configs[1]'s frame (random init, seed 1000)")
        line["config0_cpu"] = config0_cpu()
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
