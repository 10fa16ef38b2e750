"""Independent frames training concurrently in ONE process: one Python thread
and one HIP stream per frame model (1080p / 50k splats, trained state).
Reports the aggregate train-iters/s for 1, 2 and 4 frames -- the in-process
counterpart of several ranks per GPU.  ctypes drops the GIL
inside each C call and the step's host wait, so the threads' host work
interleaves while their kernels share the GPU.

    python tools/concurrent_frames.py [--frames 1 2 4] [--iters 300]
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

H, W = 1080, 1920


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--settle", type=int, default=2000)
    ap.add_argument("--splats", type=int, default=50000)
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    nmax = max(a.frames)
    models, gts, streams, its = [], [], [], []
    for f in range(nmax):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            m = make_frame_model(H, W, a.splats, dev, seed=1000 + f)
            gt = synthetic_gt(H, W, 8 + f, "cpu").to(dev)
            for it in range(1, a.settle + 1):
                m.train_iter(gt, it)
        models.append(m)
        gts.append(gt)
        streams.append(s)
        its.append(a.settle)
    torch.cuda.synchronize()

    def run(f, n, barrier, out):
        with torch.cuda.stream(streams[f]):
            barrier.wait()
            for _ in range(n):
                its[f] += 1
                models[f].train_iter(gts[f], its[f])
            torch.cuda.current_stream().synchronize()
        out[f] = time.perf_counter()

    for k in a.frames:
        barrier = threading.Barrier(k + 1)
        out = {}
        th = [threading.Thread(target=run, args=(f, a.iters, barrier, out)) for f in range(k)]
        for t in th:
            t.start()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        barrier.wait()
        for t in th:
            t.join()
        el = max(out.values()) - t0
        fused = all(models[f].fused_steps > 0 for f in range(k))
        print(json.dumps({"frames": k, "train_iters_per_s": round(k * a.iters / el, 1),
                          "us_per_iter_per_frame": round(1e6 * el / a.iters, 2),
                          "fused": fused}), flush=True)


if __name__ == "__main__":
    main()
