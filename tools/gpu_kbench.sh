#!/bin/bash
# kbench timing + rocprof kernel trace + PMC passes for the composite kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/kb
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py "$@" > $OUT/kbench.jsonl 2> $OUT/kbench.err || { echo "kbench failed"; tail -20 $OUT/kbench.err; exit 1; }
cat $OUT/kbench.jsonl
if [ -n "$KB_PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o kt --output-format csv -- python3 tools/kbench.py "$@" --iters 50 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/pmc1 -o p1 --output-format csv -- python3 tools/kbench.py "$@" --iters 20 > $OUT/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -20 $OUT/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc2 -o p2 --output-format csv -- python3 tools/kbench.py "$@" --iters 20 > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -20 $OUT/pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc3 -o p3 --output-format csv -- python3 tools/kbench.py "$@" --iters 20 > $OUT/pmc3.log 2>&1 || { echo "pmc3 failed"; tail -20 $OUT/pmc3.log; exit 1; }
echo prof-done
fi
