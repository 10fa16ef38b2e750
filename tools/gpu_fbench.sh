#!/bin/bash
# fbench (+ optional rocprofv3 kernel trace with FB_PROF=1) on the GPU box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fb
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python tools/fbench.py "$@" > $OUT/fbench.jsonl 2> $OUT/fbench.err || { echo "fbench failed"; tail -20 $OUT/fbench.err; exit 1; }
cat $OUT/fbench.jsonl
if [ -n "$FB_PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o ft --output-format csv -- python3 tools/fbench.py "$@" --iters 50 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/trace | cut -c1-150 | head -20
fi
