#!/bin/bash
# One-wave-per-tile training kernel: fused-step tests + frozen timing vs band.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3r; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_train_fused.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave or band" > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for k in band wave band wave; do
timeout -k 10 120 python tools/tbench.py --warmup 2000 --frozen 300 --tile-kernel $k >> $OUT/frozen.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/frozen.jsonl | cut -c1-200
done
