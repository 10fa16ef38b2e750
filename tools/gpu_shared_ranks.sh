#!/bin/bash
# One GPU, N bench ranks sharing it (GSVC_BENCH_SHARED_GPU=1, gloo): the
# aggregate train-iters/s and render frames/s when N independent frames train
# concurrently (frames and GOPs are independent: the video driver's
# --ranks_per_gpu), N = 1, 2, 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/shared; mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu --no-secondary > $OUT/n1.json 2> $OUT/n1.err || { tail -20 $OUT/n1.err; exit 1; }
for n in 2 4; do
  GSVC_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus $n --backend gloo --no-cpu > $OUT/n$n.json 2> $OUT/n$n.err || { tail -20 $OUT/n$n.err; exit 1; }
done
for n in 1 2 4; do
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/n$n.json') if l.startswith('{')][-1]); print('ranks_on_one_gpu=$n', d['value'], d['unit'], 'ms_per_step', d['ms_per_step'], 'render', (d.get('render') or {}).get('frames_per_s'))"
done
