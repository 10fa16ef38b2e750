#!/bin/bash
# Generic GPU-box step runner (through gpurun): optional pytest files, then
# bench.py with the given arguments, each under its own time limit; logs in
# gpurun_out/$TAG/.
#   TESTS="tests/a.py tests/b.py" BENCH="--steps 50" bash tools/gpu_run.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $OUT/tests.log | tail -30; exit 1; }
  grep -cE "PASSED" $OUT/tests.log; tail -2 $OUT/tests.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $BENCH > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
