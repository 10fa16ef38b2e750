#!/bin/bash
# Fused splat + id-order projection (knob 14 = 3) vs separate projection (0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3o; mkdir -p $OUT
for k in 0 3 0 3; do
timeout -k 10 120 python tools/tbench.py --warmup 2000 --iters 3000 --knob 14=$k --channels >> $OUT/tb.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/tb.jsonl | cut -c60-400
done
