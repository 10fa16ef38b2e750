"""Summarise rocprofv3 output for the composite kernels (bench / kbench runs).

    python tools/prof_summary.py --trace DIR [--fetch DIR] [--write DIR] [--out JSON] [--key K]

--trace  directory of a ``rocprofv3 --kernel-trace --stats`` run: prints the
         per-kernel dispatch count and average duration.
--fetch  directory of a ``--pmc FETCH_SIZE`` pass, --write of a ``--pmc
         WRITE_SIZE`` pass: per-dispatch HBM bytes of the composite kernels.
         Per /opt/skills/guides/MI355X_MICROARCH.md (HBM [CDNA4]) FETCH_SIZE
         reports half the bytes of wide streaming reads on gfx950, so it is
         doubled; WRITE_SIZE is exact for 16-B/lane stores.  rocprofv3 reports
         both in KiB.
--out    merge ``{K: {"<kernel>_bytes_per_launch": ...}}`` into this JSON file
         (profiles/pmc_traffic.json is what bench.py reads).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {"raster_sum_fwd_kernel": "rasterize_sum_forward",
           "raster_render_ids_kernel": "rasterize_sum_forward",
           "frame_project_ordered_kernel": "frame_project_ordered",
           "train_tile_wave_kernel": "train_tile",
           "train_tile_band_kernel": "train_tile",
           "raster_sum_bwd_kernel": "rasterize_sum_backward",
           "train_tile_kernel": "train_tile",
           "train_splat_kernel": "train_splat",
           "frame_project_kernel": "frame_project",
           "raster_alpha_fwd_kernel": "alpha_forward",
           "raster_alpha_bwd_kernel": "alpha_backward"}


def _short(name):
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


def _csvs(d, pattern):
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def trace_stats(d, last=0):
    rows = defaultdict(list)
    for f in _csvs(d, "*kernel_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                rows[r["Kernel_Name"]].append((int(r.get("Dispatch_Id", 0) or 0), dur))
    out = {}
    for name, ds in rows.items():
        ds.sort()
        durs = [x for _, x in (ds[-last:] if last > 0 else ds)]
        durs.sort()
        out[name] = dict(calls=len(durs), avg_us=sum(durs) / len(durs) / 1e3,
                         median_us=durs[len(durs) // 2] / 1e3, min_us=durs[0] / 1e3)
    return out


def pmc_per_launch(d, counter, last=0):
    vals = defaultdict(list)
    for f in _csvs(d, "*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                k = _short(r["Kernel_Name"])
                if k:
                    vals[k].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, v in vals.items():
        v.sort()
        v = v[-last:] if last > 0 else v
        out[k] = sum(x for _, x in v) / len(v)
    return out


def pmc_all(dirs, last=0):
    """{kernel: {counter: average per dispatch}} over every counter in the
    --pmc pass directories ``dirs`` (last > 0: over each kernel's last
    ``last`` dispatches only, e.g. the trained state of a long run)."""
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in _csvs(d, "*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = _short(r["Kernel_Name"])
                    if k:
                        vals[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]),
                                                          float(r["Counter_Value"])))
    out = {}
    for k, cs in vals.items():
        out[k] = {}
        for c, v in cs.items():
            v.sort()
            v = v[-last:] if last > 0 else v
            out[k][c] = sum(x for _, x in v) / len(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out")
    ap.add_argument("--key", default="10000")
    ap.add_argument("--pmc-dirs", nargs="*", help="print every counter per kernel")
    ap.add_argument("--last", type=int, default=0,
                    help="average each kernel's last N dispatches only (trace and PMC)")
    a = ap.parse_args()
    if a.pmc_dirs:
        print(json.dumps(pmc_all(a.pmc_dirs, a.last), indent=1))
    rec = {}
    if a.trace:
        st = trace_stats(a.trace, a.last)
        for name, s in sorted(st.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]):
            print(f"{s['calls']:6d}  avg {s['avg_us']:9.2f} us  med {s['median_us']:9.2f}  "
                  f"min {s['min_us']:9.2f}  {name[:110]}")
            k = _short(name)
            if k:
                rec.setdefault(k, {})["trace_avg_us"] = s["avg_us"]
    if a.fetch:
        for k, v in pmc_per_launch(a.fetch, "FETCH_SIZE", a.last).items():
            rec.setdefault(k, {})["fetch_bytes"] = 2.0 * v * 1024.0
    if a.write:
        for k, v in pmc_per_launch(a.write, "WRITE_SIZE", a.last).items():
            rec.setdefault(k, {})["write_bytes"] = v * 1024.0
    if rec:
        print(json.dumps(rec, indent=1))
    if a.out and rec:
        try:
            with open(a.out) as fh:
                allrec = json.load(fh)
        except (OSError, ValueError):
            allrec = {}
        entry = allrec.setdefault(a.key, {})
        for k, r in rec.items():
            if "fetch_bytes" in r and "write_bytes" in r:
                entry[f"{k}_bytes_per_launch"] = r["fetch_bytes"] + r["write_bytes"]
                entry[f"{k}_pmc"] = {x: r[x] for x in ("fetch_bytes", "write_bytes")}
            if "trace_avg_us" in r:
                entry[f"{k}_trace_avg_us"] = r["trace_avg_us"]
        entry["note"] = ("FETCH_SIZE x2 (gfx950 half-count, MI355X_MICROARCH.md HBM) + WRITE_SIZE; "
                         "KiB -> bytes; average per dispatch; trace_avg_us: rocprofv3 "
                         "--kernel-trace duration of the same command")
        with open(a.out, "w") as fh:
            json.dump(allrec, fh, indent=1)


if __name__ == "__main__":
    main()
