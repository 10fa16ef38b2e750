"""Per-run kernel durations from a rocprofv3 kernel trace: the launches of
one kernel split into runs wherever consecutive launches are more than
--gap ms apart (a tool that times several workloads in sequence, e.g.
fbench --splats 10000 50000); each run's count, mean, median and min (us).

    python tools/trace_runs.py TRACE_DIR KERNEL_SUBSTRING [--gap 2] [--min-run 50]
"""
from __future__ import annotations

import argparse
import csv
import glob
import statistics


def runs(trace: str, kernel: str, gap_ms: float = 2.0, min_run: int = 50):
    f = glob.glob(f"{trace}/**/*kernel_trace.csv", recursive=True)[0]
    hits = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                  for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"])
    out, cur, prev = [], [], None
    for s, e in hits:
        if prev is not None and s - prev > gap_ms * 1e6:
            out.append(cur)
            cur = []
        cur.append((e - s) / 1000.0)
        prev = e
    out.append(cur)
    return [r for r in out if len(r) >= min_run]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("--gap", type=float, default=2.0)
    ap.add_argument("--min-run", type=int, default=50)
    a = ap.parse_args()
    for ds in runs(a.trace, a.kernel, a.gap, a.min_run):
        print(f"{len(ds):6d}  mean {statistics.mean(ds):8.2f}  median {statistics.median(ds):8.2f}  "
              f"min {min(ds):8.2f}")


if __name__ == "__main__":
    main()
