#!/bin/bash
# One PMC pass per variant of tools/tbench.py (trained state by default):
#   bash tools/gpu_pmc_ab.sh TAG "COUNTERS" "variant args" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmcab}; shift
CTR=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CTR -d $OUT/v$i -o p --output-format csv -- python3 tools/tbench.py --warmup 2000 --iters 30 --frozen 40 $v > $OUT/v$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/v$i.log; exit 1; }
  echo "variant $i: $v"
  python3 tools/prof_summary.py --pmc-dirs $OUT/v$i --last 20 | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k: round(v) for k, v in d.get('train_tile', {}).items()}))"
done
