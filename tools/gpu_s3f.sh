#!/bin/bash
# Render at trained density: per-mode frame times and per-wave stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3f; mkdir -p $OUT
timeout -k 10 200 python tools/fbench.py --splats 50000 --trained 2000 --modes 2 1 --knob 15 1 > $OUT/fbench.jsonl 2> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
cat $OUT/fbench.jsonl
