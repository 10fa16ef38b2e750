#!/bin/bash
# The one GPU-box runner (through gpurun): runs each step under its own time
# limit, logs it to gpurun_out/$TAG/<name>.log, stops at the first failure.
#
#   gpurun -- bash tools/gpu_steps.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
#
# e.g.
#   bash tools/gpu_steps.sh r03a \
#     'tests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
#     'bench|500|python bench.py'
# A step's command runs through bash from the repo root; $OUT is its log dir.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
export OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc in $(( $(date +%s) - t0 )) s"
  tail -n ${TAIL:-4} "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then
    echo "step $name failed (rc=$rc); stopping"
    exit $rc
  fi
done
