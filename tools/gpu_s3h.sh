#!/bin/bash
# Composite crossover at high density (bigger splats).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3h; mkdir -p $OUT
for cs in 2 3 5; do
timeout -k 10 200 python tools/fbench.py --splats 50000 100000 --chol-scale $cs --modes 2 1 >> $OUT/fbench_dense.jsonl 2> $OUT/fbench.err || { tail -20 $OUT/fbench.err; exit 1; }
done
cut -c1-110 $OUT/fbench_dense.jsonl
