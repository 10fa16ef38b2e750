#!/bin/bash
# Alpha path timing + kernel trace at 1080p.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/alpha; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/alphabench.py > $OUT/alphabench.jsonl 2> $OUT/a.err || { tail -20 $OUT/a.err; exit 1; }
cat $OUT/alphabench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o a --output-format csv -- python3 tools/alphabench.py --splats 50000 --calls 100 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12 | cut -c1-200
