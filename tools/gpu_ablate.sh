#!/bin/bash
# Tile-kernel cost breakdown at trained density: frozen gradient-only steps
# with the band kernel's diagnostic bits (knob 13) set after the warmup.
# Usage: gpu_ablate.sh TAG "bits..." [extra tbench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ablate}; BITS=${2:-"0 1 2 4 8 16 32 6"}; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for b in $BITS; do
  timeout -k 10 120 python tools/tbench.py --warmup 2000 --frozen 300 --knob-after 13=$b "$@" >> $OUT/ablate.jsonl 2>> $OUT/ablate.err || { echo "bits $b failed"; tail -20 $OUT/ablate.err; exit 1; }
  tail -1 $OUT/ablate.jsonl
done
