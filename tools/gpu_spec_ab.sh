#!/bin/bash
# Composite at 1080p / 10k: speculative slab records per tile (knob 10 = 8, 4,
# 2) -- kernel time (trace) and HBM reads (FETCH_SIZE x 2, gfx950) per launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/spec_ab; mkdir -p $OUT
export TMPDIR=/tmp
for v in 8 4 2 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$v -o t --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 200 --knob 10 $v > $OUT/t$v.log 2>&1 || { tail -20 $OUT/t$v.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/f$v -o f --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 200 --knob 10 $v > $OUT/f$v.log 2>&1 || { tail -20 $OUT/f$v.log; exit 1; }
  python3 - "$OUT" "$v" <<'PY'
import csv, glob, sys
out, v = sys.argv[1], sys.argv[2]
tr = glob.glob(f"{out}/t{v}/**/*kernel_trace.csv", recursive=True)[0]
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tr))
        if "raster_sum_fwd" in r["Kernel_Name"]]
pc = glob.glob(f"{out}/f{v}/**/*counter_collection.csv", recursive=True)[0]
fs = [float(r["Counter_Value"]) for r in csv.DictReader(open(pc))
      if "raster_sum_fwd" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
last = durs[-100:]
print(f"spec_slots={v} composite_us={sum(last) / len(last) / 1e3:.2f} "
      f"fetch_MB={2 * 1024 * sum(fs[-100:]) / len(fs[-100:]) / 1e6:.2f} launches={len(durs)}")
PY
done
