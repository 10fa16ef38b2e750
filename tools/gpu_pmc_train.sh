#!/bin/bash
# PMC counters of the fused training step's kernels (through gpurun): one
# rocprofv3 --pmc pass per counter group, each under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o p --output-format csv -- python3 tools/tbench.py --iters 20 --warmup 5 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/prof_summary.py --pmc-dirs $OUT/p* > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt | head -60
