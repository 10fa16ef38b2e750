#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_alpha_path.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python tools/alphabench.py > $OUT/alphabench.jsonl 2> $OUT/a.err || { tail -20 $OUT/a.err; exit 1; }
cat $OUT/alphabench.jsonl
