#!/bin/bash
# Bench + rocprofv3 kernel trace on the GPU box (run through gpurun).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-secondary --steps 100 --warmup 10 > $OUT/prof_bench.log 2>&1 || { echo "rocprof failed rc=$?"; tail -30 $OUT/prof_bench.log; exit 1; }
find $OUT/prof -name "*stats*" | head
