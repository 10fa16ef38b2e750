#!/bin/bash
# Grouped forward (knob 15): training GPU tests + tbench A/B + frozen ablation A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_train_fused.py tests/test_frame_train.py tests/test_train_trajectory.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for k in 0 1 0 1; do
timeout -k 10 120 python tools/tbench.py --warmup 2000 --frozen 300 --knob-after 15=$k >> $OUT/frozen.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/frozen.jsonl | cut -c1-300
done
timeout -k 10 120 python tools/tbench.py --warmup 2000 --iters 2000 --channels >> $OUT/tb.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/tb.jsonl | cut -c1-400
