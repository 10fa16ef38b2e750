#!/bin/bash
# Video encode throughput on ONE GPU: the same 8-frame synthetic 1080p video
# (GOPs 1-4 and 5-8, 50k splats, ITERS iterations per frame) trained by 1 rank,
# then by 2 and 4 ranks sharing the GPU (--ranks_per_gpu, gloo collectives).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/video_rpg; mkdir -p $OUT
ITERS=${ITERS:-2000}
COMMON="--synthetic 8 --k_frames 1,3,5,7 --iterations $ITERS --num_points 50000"
run() {  # ranks
  local n=$1 t0 t1
  t0=$(date +%s.%N)
  if [ $n = 1 ]; then
    timeout -k 10 300 python -m gsvc_amd.video $COMMON --root /tmp/vr1 > $OUT/r$n.log 2>&1 || { tail -20 $OUT/r$n.log; return 1; }
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) -m gsvc_amd.video $COMMON --ranks_per_gpu $n --root /tmp/vr$n > $OUT/r$n.log 2>&1 || { tail -20 $OUT/r$n.log; return 1; }
  fi
  t1=$(date +%s.%N)
  echo "ranks_on_one_gpu=$n wall_s=$(python3 -c "print(round($t1 - $t0, 2))") $(grep '^{' $OUT/r$n.log | tail -1 | cut -c1-300)"
}
run 1 && run 2 && run 4
