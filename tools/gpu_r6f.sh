set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; OUT=gpurun_out/r6f; mkdir -p $OUT
for v in 1 2 4 8 16 3 9 13 18; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k$v -o a --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 400 --knob 36 $v > $OUT/k$v.log 2>&1 || exit 1
  echo "== 36=$v"; python3 tools/trace_runs.py $OUT/k$v raster_render_ids
done
