set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; OUT=gpurun_out/r6g; mkdir -p $OUT
for rep in 1 2; do
for v in 1 2 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k${v}_$rep -o a --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 400 --knob 38 $v > $OUT/k${v}_$rep.log 2>&1 || exit 1
  grep identical $OUT/k${v}_$rep.log | cut -c1-200
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t${v}_$rep -o a --output-format csv -- python3 tools/fbench.py --splats 50000 --trained 2000 --iters 400 --knob 38 $v > $OUT/t${v}_$rep.log 2>&1 || exit 1
  grep identical $OUT/t${v}_$rep.log | cut -c1-200
done; done
python3 tools/knob_ab.py raster_ $OUT/k* $OUT/t*
