"""Per (kernel, grid) average durations from a rocprofv3 kernel-trace CSV dir.

    python tools/trace_by_grid.py <trace dir> [kernel substring]
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if sub not in n:
            continue
        key = (n.split("(")[0][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(acc.items()):
    v.sort()
    print(f"{k[0]:60s} grid {k[1]:>8s} {k[2]:>4s} {k[3]:>3s}  n={len(v):4d}  avg {sum(v) / len(v):8.1f} us"
          f"  med {v[len(v) // 2]:8.1f}")
