#!/bin/bash
# Prune kernel: GPU parity tests, then the cost against the torch sequence.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prune
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_prune.py tests/test_train_fused.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
grep -c PASSED $OUT/t.log; tail -1 $OUT/t.log
timeout -k 10 200 python tools/prunebench.py > $OUT/bench.jsonl 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o pr --output-format csv -- python3 tools/prunebench.py --iters 20 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/trace | cut -c1-150 | head -16
