set -o pipefail
OUT=gpurun_out/dab; mkdir -p $OUT
for rep in 1 2; do
  for v in s0 cap wg cur; do
    GSVC_DIAG=1 GSVC_DIAG_LIB=$PWD/gsvc_amd/lib/alt/$v/libgsvc_amd_diag.so timeout -k 10 200 python tools/tbench.py --state profiles/r05/overflow/textured_frame116.npz:116 --channels --iters 300 > $OUT/${v}_$rep.log 2>&1 || { echo "fail $v"; tail -3 $OUT/${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"iters_per_s": [0-9.]*' $OUT/${v}_$rep.log) $(grep -o '"train_tile": [0-9.]*' $OUT/${v}_$rep.log)"
  done
done
