#!/bin/bash
# Batched decode: knob A/B + kernel trace (LDS / scratch per dispatch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/vbench.py --knob 15 1 > $OUT/vbench.jsonl 2> $OUT/v.err || { tail -20 $OUT/v.err; exit 1; }
cat $OUT/vbench.jsonl | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o v --output-format csv -- python3 tools/vbench.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
print(list(rows[0].keys()))
seen=collections.OrderedDict()
for r in rows:
    k=r['Kernel_Name'][:60]
    if k not in seen: seen[k]=(r.get('LDS_Block_Size'),r.get('Scratch_Size'),r.get('VGPR_Count'),r.get('Workgroup_Size'))
for k,v in seen.items(): print(k,v)
PY
