#!/bin/bash
# Same-box A/B of the alpha backward's reductions (knob 9: 0 = DPP row sums,
# 1 = shuffle butterflies): kernel trace per variant, interleaved twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/alpha_ab; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for k in 0 1; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k${k}_$rep -o a --output-format csv -- python3 tools/alphabench.py --splats 50000 --calls 100 --knob 9=$k > $OUT/k${k}_$rep.log 2>&1 || { tail -20 $OUT/k${k}_$rep.log; exit 1; }
    f=$(find $OUT/k${k}_$rep -name "*kernel_stats.csv" | head -1)
    echo "knob9=$k rep$rep $(grep raster_alpha_bwd "$f" | awk -F'",' '{print $2}' | cut -d, -f1-4) | $(grep '{' $OUT/k${k}_$rep.log | tail -1)"
  done
done
