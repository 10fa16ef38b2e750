#!/bin/bash
# Quick training-step check on the GPU box: tbench (with per-tile stamps)
# and a kernel trace of it; gpurun_out/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tb}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 200 python tools/tbench.py --stamps "$@" > $OUT/tbench.jsonl 2> $OUT/tbench.err || { echo "tbench failed"; tail -20 $OUT/tbench.err; exit 1; }
cat $OUT/tbench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o tt --output-format csv -- python3 tools/tbench.py --iters 50 "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/trace > $OUT/trace_summary.txt
cut -c1-130 $OUT/trace_summary.txt | head -6
