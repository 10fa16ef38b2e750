#!/bin/bash
# Training tests + frozen tile-kernel timing (current tree).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/${TAG:-s3d}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_train_fused.py tests/test_frame_train.py tests/test_train_trajectory.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for k in ${KNOBS:-0 0}; do
timeout -k 10 120 python tools/tbench.py --warmup 2000 --frozen 300 --knob-after $k >> $OUT/frozen.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/frozen.jsonl | cut -c1-300
done
