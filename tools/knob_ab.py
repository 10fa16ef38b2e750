"""Summarise fbench knob A/Bs traced by rocprofv3: each trace dir holds one
fbench run whose first half of the kernel's launches are the default pass and
whose second half the --knob pass (fbench prints whether the images matched).

    python tools/knob_ab.py KERNEL_SUBSTRING DIR [DIR ...]
"""
from __future__ import annotations

import csv
import glob
import statistics
import sys


def halves(d, kernel):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    h = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
               for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"])
    t = [(e - s) / 1000.0 for s, e in h]
    return t


def main():
    kernel = sys.argv[1]
    for d in sys.argv[2:]:
        if not glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
            continue
        f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        names = [r["Kernel_Name"] for r in rows if any(k in r["Kernel_Name"] for k in kernel.split(","))]
        t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rows
             if any(k in r["Kernel_Name"] for k in kernel.split(","))]
        # consecutive runs of one kernel name (a variant switch changes the kernel)
        runs, cur, nm = [], [], None
        for n, x in zip(names, t):
            if n != nm and cur:
                runs.append((nm, cur))
                cur = []
            nm = n
            cur.append(x)
        runs.append((nm, cur))
        for nm, r in runs:
            if len(r) >= 50:
                r = r[20:]
                print(f"{d.split('/')[-1]:>12}  n={len(r):5d}  mean {statistics.mean(r):7.2f}  "
                      f"median {statistics.median(r):7.2f}  {nm[:60]}")


if __name__ == "__main__":
    main()
