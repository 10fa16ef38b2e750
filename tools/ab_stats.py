"""Average duration per kernel and variant of a tools/ab_builds.sh or gpu.sh
A/B run: python tools/ab_stats.py gpurun_out/TAG [name-filter]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    fs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if filt in r["Name"]:
                print(f"{os.path.basename(d.rstrip('/')):12s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.2f} us  {r['Name'][:80]}")
