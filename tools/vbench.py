"""Batched (GOP) render throughput, bench.py's video_decode, with an optional
A/B pass of gsvc_debug_set(KEY, VALUE).

    python tools/vbench.py [--frames 8] [--knob 2 8]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# A/B knobs and timestamped variants: the diagnostic library (gsvc_amd/_lib.py)
os.environ.setdefault("GSVC_DIAG", "1")

import torch  # noqa: E402

import bench  # noqa: E402
from gsvc_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, nargs="+", default=[8])
    ap.add_argument("--knob", type=int, nargs=2, action="append", default=[])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = L.load()
    for f in a.frames:
        for kv in [None] + a.knob:
            if kv:
                if lib.gsvc_debug_set(kv[0], kv[1]) < 0:
                    raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")
            r = bench.video_decode(dev, frames=f)
            if kv:
                lib.gsvc_debug_set(kv[0], 0)
            print(json.dumps(dict(frames=f, knob=kv, fps=round(r["frames_per_s"]),
                                  kernel_us=r["roofline"]["avg_kernel_us"],
                                  frac=r["roofline"]["frac"])), flush=True)


if __name__ == "__main__":
    main()
