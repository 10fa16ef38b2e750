#!/bin/bash
# VALU / LDS instruction counts of the composite at trained 1080p / 50k (the
# render_50000 dispatches of tools/pmc_workloads.py train50k), last 50 launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/pmc_comp; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES -d $OUT/p -o p --output-format csv -- python3 tools/pmc_workloads.py train50k > $OUT/p.log 2>&1 || { tail -20 $OUT/p.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, json, collections
f = glob.glob(f"{sys.argv[1]}/p/**/*counter_collection.csv", recursive=True)[0]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    for key in ("raster_sum_fwd", "train_tile_band"):
        if key in r["Kernel_Name"]:
            by[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: round(sum(v[-50:]) / len(v[-50:])) for c, v in d.items()} for k, d in by.items()}
print(json.dumps(out))
PY
