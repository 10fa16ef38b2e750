#!/bin/bash
# Round-end evidence on the GPU box: the whole GPU suite, smoke(), the default
# bench.py line, then the kernel trace and the FETCH_SIZE / WRITE_SIZE passes of
# the bench command (tools/gpu_bench_prof.sh), all into gpurun_out/final/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
PARGS="--no-cpu --no-secondary --steps 100 --warmup 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py $PARGS > $OUT/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf -o f --output-format csv -- python3 bench.py $PARGS > $OUT/pmcf.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmcf.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw -o w --output-format csv -- python3 bench.py $PARGS > $OUT/pmcw.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmcw.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/prof --fetch $OUT/pmcf --write $OUT/pmcw --out $OUT/pmc_traffic.json --key 10000 > $OUT/prof_summary.txt
head -6 $OUT/prof_summary.txt | cut -c1-150
