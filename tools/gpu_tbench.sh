#!/bin/bash
# tbench + rocprofv3 kernel trace of the training iteration (through gpurun).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tb
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python tools/tbench.py "$@" > $OUT/tbench.jsonl 2> $OUT/tbench.err || { echo "tbench failed"; tail -20 $OUT/tbench.err; exit 1; }
timeout -k 10 300 python tools/tbench.py --op-by-op "$@" >> $OUT/tbench.jsonl 2>> $OUT/tbench.err || { echo "tbench failed"; tail -20 $OUT/tbench.err; exit 1; }
cat $OUT/tbench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o tt --output-format csv -- python3 tools/tbench.py "$@" --iters 50 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/trace | cut -c1-150 | head -30
