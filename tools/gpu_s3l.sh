#!/bin/bash
# Projection insertion batching: training tests + projection stamps/timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_train_fused.py tests/test_frame_train.py tests/test_train_trajectory.py tests/test_gpu_sync_free.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python tools/tbench.py --warmup 2000 --iters 2000 --channels --proj-stamps > $OUT/tb.jsonl 2> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
cut -c1-400 $OUT/tb.jsonl
