#!/bin/bash
# Sparse composite: list threshold A/B (knob 15 = v: lists above v - 1 entries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sync_free.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python tools/fbench.py --splats 50000 --trained 2000 --modes 1 --knob 15 1 --knob 15 5 --knob 15 13 > $OUT/fbench_trained.jsonl 2> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
timeout -k 10 200 python tools/fbench.py --splats 10000 50000 --modes 1 --knob 15 1 --knob 15 5 --knob 15 13 > $OUT/fbench_init.jsonl 2>> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
cut -c1-110 $OUT/fbench_trained.jsonl $OUT/fbench_init.jsonl
timeout -k 10 200 python tools/vbench.py > $OUT/vbench.jsonl 2>> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
tail -3 $OUT/vbench.jsonl | cut -c1-200
