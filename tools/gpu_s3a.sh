#!/bin/bash
# Ablation breakdown of the current band kernel + trained dump + projection stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_ablate.sh s3a "0 2 4 6 8 16 32" || exit 1
timeout -k 10 200 python tools/dump_trained.py --out gpurun_out/s3a/trained_50k.npz > gpurun_out/s3a/dump.log 2>&1 || { tail gpurun_out/s3a/dump.log; exit 1; }
timeout -k 10 120 python tools/tbench.py --warmup 2000 --iters 50 --proj-stamps --stamps > gpurun_out/s3a/projstamps.log 2>&1 || { tail gpurun_out/s3a/projstamps.log; exit 1; }
tail -30 gpurun_out/s3a/projstamps.log
