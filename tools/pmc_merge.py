"""Merge tools/gpu.sh pmc_final's counter passes into the pmc_valu.json that
bench.py reads (profiles/pmc_valu.json): per kernel key the mean of its last
50 dispatches of each counter.

    python tools/pmc_merge.py gpurun_out/TAG > profiles/pmc_valu.json
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import subprocess
import sys

# (workload dir, kernel-name substring) -> bench.py key
KEYS = {("train50k", "train_tile_band"): "train_tile",
        ("train50k", "raster_render_ids"): "render_50000",
        ("render10k", "raster_render_ids"): "render_10000",
        ("train50k", "train_splat"): "train_splat"}


def main():
    out = sys.argv[1]
    res = {}
    for (wl, kern), key in KEYS.items():
        d = collections.defaultdict(list)
        name = None
        for sub in ("valu", "sq"):
            for f in glob.glob(f"{out}/{wl}/{sub}/**/*counter_collection.csv", recursive=True):
                for r in csv.DictReader(open(f)):
                    if kern in r["Kernel_Name"]:
                        name = r["Kernel_Name"].split("(")[0]
                        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if not d:
            continue
        e = {"kernel": name}
        for c, v in sorted(d.items()):
            e[c] = round(sum(v[-50:]) / len(v[-50:]))
        rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
        e["source"] = (f"rocprofv3 --pmc of tools/pmc_workloads.py {wl}, the library of commit {rev} "
                       f"(+ working tree), last 50 dispatches (tools/gpu.sh pmc_final)")
        res[key] = e
    res["note"] = ("SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; a wave64 VALU "
                   "instruction issues over 2 cycles (MI355X_MICROARCH.md); bench.py's valu roofline: "
                   "SQ_INSTS_VALU x 2 cycles against 1024 SIMDs x 2.4 GHz")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
