"""The op path's image layout A/B in ONE process (host noise shared):
GSVC_OP_PLANAR=1 (channel planes, the default) against =0 (contiguous
[H, W, 3]), alternated ``--reps`` times, each block ``--calls`` forward +
backward calls (GSVC's forward, MSE, backward) and as many forwards, at the
bench's trained 1080p / 50k state.  Prints one JSON line per block and the
medians.

    python tools/planar_ab.py [--reps 6] [--calls 200]
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from opprof import calls, model_at  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(REPO, "tests/golden/train_state_1080p_n50k.npz"))
    from gsvc_amd.frame import synthetic_gt
    H, W = 1080, 1920
    m = model_at(H, W, int(z["n"]), dev, {k: z[k] for k in z.files if k.startswith("state_")})
    gt = synthetic_gt(H, W, int(z["gt_seed"]), dev)
    fns = calls(m, gt)

    def timed(fn, k):
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.05:
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    res = {"1": {"fwd": [], "fwd_bwd": []}, "0": {"fwd": [], "fwd_bwd": []}}
    for rep in range(a.reps):
        for lay in ("1", "0"):
            os.environ["GSVC_OP_PLANAR"] = lay
            f = timed(fns["fwd"], a.calls)
            fb = timed(fns["fwd_bwd"], a.calls)
            res[lay]["fwd"].append(f)
            res[lay]["fwd_bwd"].append(fb)
            print(json.dumps(dict(rep=rep, planar=lay, fwd_us=round(f, 1), fwd_bwd_us=round(fb, 1))),
                  flush=True)
    print(json.dumps({("planar" if k == "1" else "hwc"): {q: round(statistics.median(v), 1)
                                                          for q, v in d.items()}
                      for k, d in res.items()}))


if __name__ == "__main__":
    main()
