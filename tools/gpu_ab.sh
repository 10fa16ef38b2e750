#!/bin/bash
# A/B of the fused training step on the GPU box: optional GPU tests ($TESTS,
# pytest paths), then tools/tbench.py --channels once per variant (each
# variant a quoted string of tbench arguments, e.g. "--knob 4=2").
# Outputs in gpurun_out/$TAG/.
#   TESTS="tests/test_train_fused.py" bash tools/gpu_ab.sh TAG "" "--knob 4=4"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
for v in "$@"; do
  timeout -k 10 200 python tools/tbench.py --channels $v >> $OUT/ab.jsonl 2> $OUT/ab.err || { echo "tbench failed ($v)"; tail -20 $OUT/ab.err; exit 1; }
  tail -1 $OUT/ab.jsonl
done
