"""Where the unchanged-caller op path spends its time (bench.py's op_path):
GaussianVideoFrame with fused_train / fused_render off -- GSVC's own op
sequence over the gsplat drop-in -- at the bench's trained 1080p / 50k state
(tests/golden/train_state_1080p_n50k.npz) and at a 16x16 / 16-splat frame
(host cost alone).  Prints wall time per call for forward, forward +
backward, no-grad render and train_iter, then a cProfile of forward +
backward and a torch.profiler table (host time per op and per autograd node,
so the drop-in's own share -- project / rasterize forward and their backward
nodes -- reads apart from the caller's ops).  Run it under
``rocprofv3 --kernel-trace --stats`` for the kernels.

    python tools/opprof.py [--calls 200] [--no-profile] [--only 1080p_50k_trained]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def model_at(H, W, n, dev, state=None):
    from gsvc_amd.frame import make_frame_model
    m = make_frame_model(H, W, n, dev, seed=0, fused_train=False, fused_render=False)
    if state is not None:
        with torch.no_grad():
            for k in ("_xyz", "_cholesky", "_features_dc"):
                getattr(m, k).copy_(torch.from_numpy(state["state_" + k]))
    return m


def timed(fn, k, w=20):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6


def calls(m, gt):
    def fwd():
        m.forward()

    def fwd_bwd():
        for p in (m._xyz, m._cholesky, m._features_dc):
            p.grad = None
        img = m.forward()["render"]
        F.mse_loss(img.squeeze(0), gt.squeeze(0)).backward()

    def render():
        with torch.no_grad():
            m.forward()

    it = [0]

    def train():
        it[0] += 1
        m.train_iter(gt, it[0])
    return dict(fwd=fwd, fwd_bwd=fwd_bwd, render=render, train=train)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--only", default=None, help="run one size: 1080p_50k_trained or tiny_16x16_16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from gsvc_amd.frame import synthetic_gt
    z = np.load(os.path.join(REPO, "tests", "golden", "train_state_1080p_n50k.npz"))
    res = {}
    for tag, (H, W, n, st) in {"1080p_50k_trained": (1080, 1920, int(z["n"]), z),
                               "tiny_16x16_16": (16, 16, 16, None)}.items():
        if a.only and tag != a.only:
            continue
        m = model_at(H, W, n, dev, st)
        gt = synthetic_gt(H, W, 8, "cpu").to(dev)
        res[tag] = {k: round(timed(f, a.calls), 1) for k, f in calls(m, gt).items()}
    print(json.dumps(res), flush=True)
    if a.no_profile:
        return
    m = model_at(1080, 1920, int(z["n"]), dev, z)
    gt = synthetic_gt(1080, 1920, 8, "cpu").to(dev)
    fb = calls(m, gt)["fwd_bwd"]
    timed(fb, 20)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.calls):
        fb()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue()[:5000])
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(a.calls):
            fb()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30,
                                    max_name_column_width=60), flush=True)


if __name__ == "__main__":
    main()
