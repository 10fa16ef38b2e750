#!/bin/bash
# A/B of PRODUCT-library builds through bench.py (AB_SECONDARY= for the
# secondary workloads too: op path, renders, alpha): the in-tree library and every
# gsvc_amd/lib/alt/<v>/libgsvc_amd.so (tools/build_alt.py --product) swapped in
# turn into gsvc_amd/lib/libgsvc_amd.so on the GPU box's scratch copy, REPS
# interleaved rounds; each run's bench line (value, tile / splat kernel us).
#
#   gpurun -- bash tools/ab_product.sh TAG [REPS] [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
REPS=${2:-2}
shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
LIB=gsvc_amd/lib/libgsvc_amd.so
cp $LIB $OUT/cur.so
for rep in $(seq 1 $REPS); do
  for d in cur gsvc_amd/lib/alt/*/; do
    if [ "$d" = cur ]; then v=cur; src=$OUT/cur.so; else v=$(basename "$d"); src=$d/libgsvc_amd.so; fi
    [ -f "$src" ] || continue
    cp "$src" $LIB
    timeout -k 10 300 python -u bench.py --no-cpu ${AB_SECONDARY:---no-secondary} "$@" > "$OUT/${v}_$rep.log" 2>&1 \
      || { echo "variant $v failed"; tail -5 "$OUT/${v}_$rep.log"; cp $OUT/cur.so $LIB; exit 1; }
    python3 - "$OUT/${v}_$rep.log" "$v" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
k = d.get("kernels", {})
print(f"{sys.argv[2]:>10}  {d['value']:9.1f} it/s  tile {d['roofline']['avg_kernel_us']:6.2f}  "
      f"splat {k.get('train_splat', {}).get('avg_kernel_us', 0):6.2f} us", end="")
op = d.get("op_path")
if op:
    ok = op.get("kernels", {})
    print(f"  op fwd {op['fwd_us']:6.1f} fwd+bwd {op['fwd_bwd_us']:6.1f}  op kernels fwd "
          f"{ok.get('raster_sum_fwd', {}).get('avg_kernel_us', 0):6.2f} bwd "
          f"{ok.get('raster_sum_bwd', {}).get('avg_kernel_us', 0):6.2f}", end="")
for key in ("render", "render_10k"):
    r = d.get(key)
    if r:
        print(f"  {key} {r['frames_per_s']:8.0f} fps {r['roofline']['avg_kernel_us']:6.2f} us", end="")
print()
PY
  done
done
cp $OUT/cur.so $LIB
