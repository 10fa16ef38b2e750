#!/bin/bash
# Kernel-trace + HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) of
# the bench's workloads (tools/pmc_workloads.py) on the GPU box; summaries of
# each kernel's last 50 dispatches into gpurun_out/$TAG/pmc_traffic.json (keys
# train_50000, render_50000, render_10000 as bench.py reads them).
#   bash tools/gpu_bench_pmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-benchpmc}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for wl in train50k render10k; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$wl/trace -o t --output-format csv -- python3 tools/pmc_workloads.py $wl > $OUT/$wl.trace.log 2>&1 || { echo "trace $wl failed"; tail -5 $OUT/$wl.trace.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/$wl/fetch -o f --output-format csv -- python3 tools/pmc_workloads.py $wl > $OUT/$wl.fetch.log 2>&1 || { echo "fetch $wl failed"; tail -5 $OUT/$wl.fetch.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/$wl/write -o w --output-format csv -- python3 tools/pmc_workloads.py $wl > $OUT/$wl.write.log 2>&1 || { echo "write $wl failed"; tail -5 $OUT/$wl.write.log; exit 1; }
done
for key in train_50000 render_50000; do
  python3 tools/prof_summary.py --trace $OUT/train50k/trace --fetch $OUT/train50k/fetch --write $OUT/train50k/write --last 50 --out $OUT/pmc_traffic.json --key $key > $OUT/$key.txt
done
python3 tools/prof_summary.py --trace $OUT/render10k/trace --fetch $OUT/render10k/fetch --write $OUT/render10k/write --last 50 --out $OUT/pmc_traffic.json --key render_10000 > $OUT/render_10000.txt
cat $OUT/train_50000.txt | cut -c1-150 | head -12
cat $OUT/pmc_traffic.json
