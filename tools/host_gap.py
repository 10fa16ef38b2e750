"""Host-side critical path of the fused training loop on the GPU box: from
BoundStep.result() returning (the loss word seen) to the next step's C call
entering and returning (the tile kernel submitted).  Trains the bench's
1080p / 50k frame (seed 1000) --settle iterations, then times --steps.

  python tools/host_gap.py [--settle 2000] [--steps 400]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settle", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    from gsvc_amd import train as T
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    dev = torch.device("cuda:0")
    m = make_frame_model(1080, 1920, 50000, dev, seed=1000)
    gt = synthetic_gt(1080, 1920, 8, "cpu").to(dev)
    it = 0
    for _ in range(a.settle):
        it += 1
        m.train_iter(gt, it)
    torch.cuda.synchronize()
    rec = {"res_end": [], "call_begin": [], "call_end": [], "res_begin": []}
    orig_result, orig_call = T.BoundStep.result, T.BoundStep._call

    def result(self):
        rec["res_begin"].append(time.perf_counter())
        r = orig_result(self)
        rec["res_end"].append(time.perf_counter())
        return r

    def call(self, ws, lib, gt, flags):
        rec["call_begin"].append(time.perf_counter())
        r = orig_call(self, ws, lib, gt, flags)
        rec["call_end"].append(time.perf_counter())
        return r

    T.BoundStep.result, T.BoundStep._call = result, call
    t0 = time.perf_counter()
    for _ in range(a.steps):
        it += 1
        m.train_iter(gt, it)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    T.BoundStep.result, T.BoundStep._call = orig_result, orig_call
    n = min(len(rec["res_end"]), len(rec["call_begin"])) - 1
    # steps without a rebuild: one _call per step
    gaps = [rec["call_begin"][k + 1] - rec["res_end"][k] for k in range(n)]
    calls = [e - b for b, e in zip(rec["call_begin"], rec["call_end"])]
    waits = [e - b for b, e in zip(rec["res_begin"], rec["res_end"])]
    pre = [rec["res_begin"][k] - rec["call_end"][k] for k in range(n)]
    med = lambda v: sorted(v)[len(v) // 2] * 1e6
    print(json.dumps({"us_per_step": round(wall * 1e6, 2), "calls": len(calls), "steps": a.steps,
                      "python_result_to_next_call_us": round(med(gaps), 2),
                      "c_call_us": round(med(calls), 2),
                      "after_call_to_wait_us": round(med(pre), 2),
                      "wait_us": round(med(waits), 2)}))


if __name__ == "__main__":
    main()
