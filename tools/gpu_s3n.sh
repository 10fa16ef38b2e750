#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3n; mkdir -p $OUT
timeout -k 10 120 python tools/tbench.py --warmup 2000 --iters 50 --proj-stamps > $OUT/ps.log 2>&1 || { tail -20 $OUT/ps.log; exit 1; }
grep proj_stamps $OUT/ps.log
