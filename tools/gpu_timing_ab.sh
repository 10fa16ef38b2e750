#!/bin/bash
# bench.py with the composite kernel timed by dispatch-carried events vs marker
# events around the launch (same frame loop), then a kernel trace of the first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tab
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for how in dispatch marker dispatch marker; do
timeout -k 10 200 python bench.py --no-cpu --no-secondary --timing $how >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "bench $how failed"; tail -20 $OUT/ab.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/tab/ab.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(r["timing"][:40], d["value"], r["avg_kernel_us"], r["frac"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o tr --output-format csv -- python3 bench.py --no-cpu --no-secondary --steps 100 --warmup 10 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/trace | cut -c1-150 | head -12
tail -1 $OUT/trace.log | cut -c1-400
