#!/bin/bash
# On the GPU box (through gpurun): bench.py, then rocprofv3 kernel trace and the
# FETCH_SIZE / WRITE_SIZE passes of the same command, summarised by
# tools/prof_summary.py into gpurun_out/ (copy what is judged into profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
PARGS="--no-cpu --no-secondary --steps 100 --warmup 10 $PROF_ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py $PARGS > $OUT/prof_bench.log 2>&1 || { echo "rocprof failed rc=$?"; tail -30 $OUT/prof_bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf -o f --output-format csv -- python3 bench.py $PARGS > $OUT/pmcf.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmcf.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw -o w --output-format csv -- python3 bench.py $PARGS > $OUT/pmcw.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmcw.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/prof --fetch $OUT/pmcf --write $OUT/pmcw --out $OUT/pmc_traffic.json --key ${PROF_KEY:-10000} > $OUT/prof_summary.txt
cat $OUT/prof_summary.txt | cut -c1-160 | head -40
timeout -k 10 500 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
