"""Where a fused train_iter's wall time goes at 1080p / 50k splats: the
Python work before the step's launch (critical path after the previous
PSNR read-back), the enqueue, the work overlapped with the kernels, and the
wait.  cProfile of the Python side with --profile.

    python tools/hostprof.py [--iters 200] [--profile]
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

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--splats", type=int, default=50000)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    from gsvc_amd import train as T
    dev = torch.device("cuda:0")
    m = make_frame_model(1080, 1920, a.splats, dev, seed=7)
    gt = synthetic_gt(1080, 1920, 8, dev)
    for it in range(1, 21):
        m.train_iter(gt, it)
    torch.cuda.synchronize()
    # instrument BoundStep.launch / result
    acc = dict(launch=0.0, result=0.0, pre=0.0, mid=0.0, post=0.0)
    orig_l, orig_r = T.BoundStep.launch, T.BoundStep.result
    mark = {}

    def launch(self, *x):
        t = time.perf_counter()
        acc["pre"] += t - mark["start"]
        orig_l(self, *x)
        mark["launched"] = time.perf_counter()
        acc["launch"] += mark["launched"] - t

    def result(self):
        t = time.perf_counter()
        acc["mid"] += t - mark["launched"]
        r = orig_r(self)
        mark["waited"] = time.perf_counter()
        acc["result"] += mark["waited"] - t
        return r

    T.BoundStep.launch, T.BoundStep.result = launch, result
    t0 = time.perf_counter()
    for it in range(21, 21 + a.iters):
        mark["start"] = time.perf_counter()
        m.train_iter(gt, it)
        acc["post"] += time.perf_counter() - mark["waited"]
    total = (time.perf_counter() - t0) / a.iters * 1e6
    T.BoundStep.launch, T.BoundStep.result = orig_l, orig_r
    print(json.dumps(dict(us_per_iter=round(total, 2),
                          launch_us=round(acc["launch"] / a.iters * 1e6, 2),
                          wait_us=round(acc["result"] / a.iters * 1e6, 2),
                          other_python_us=round(total - (acc["launch"] + acc["result"]) / a.iters * 1e6, 2),
                          pre_launch_us=round(acc["pre"] / a.iters * 1e6, 2),
                          launch_to_wait_us=round(acc["mid"] / a.iters * 1e6, 2),
                          post_wait_us=round(acc["post"] / a.iters * 1e6, 2))),
          flush=True)
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        for it in range(21 + a.iters, 21 + 2 * a.iters):
            m.train_iter(gt, it)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(20)
        print(s.getvalue()[:5000])


if __name__ == "__main__":
    main()
