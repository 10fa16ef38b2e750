#!/bin/bash
# Staged next-frame projection (knob 14 = 0) vs the separate projection (= 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for k in 0 1 0 1; do
timeout -k 10 120 python tools/tbench.py --warmup 2000 --iters 3000 --knob 14=$k --channels >> $OUT/tb.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/tb.jsonl | cut -c60-400
done
