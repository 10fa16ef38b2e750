#!/bin/bash
# Full GPU suite + composite modes at trained and random-init density.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python tools/fbench.py --splats 50000 --trained 2000 --modes 2 1 > $OUT/fbench_trained.jsonl 2> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
cat $OUT/fbench_trained.jsonl
timeout -k 10 200 python tools/fbench.py --splats 10000 20000 30000 50000 100000 --modes 2 1 > $OUT/fbench_init.jsonl 2>> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
cut -c1-120 $OUT/fbench_init.jsonl
