#!/bin/bash
# A/B of diagnostic-library BUILDS (not knobs): every variant directory
# gsvc_amd/lib/alt/<v>/ holding a libgsvc_amd_diag.so is run twice,
# interleaved, under rocprofv3 --kernel-trace --stats (GSVC_DIAG_LIB picks the
# build; the tool must load the diagnostic library, e.g. tools/alphabench.py).
#
#   gpurun -- bash tools/ab_builds.sh TAG python3 tools/alphabench.py --splats 50000 --calls 100
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
  for d in gsvc_amd/lib/alt/*/; do
    v=$(basename "$d")
    echo "== $v rep $rep"
    GSVC_DIAG=1 GSVC_DIAG_LIB=$R/$d/libgsvc_amd_diag.so timeout -k 10 200 \
      rocprofv3 --kernel-trace --stats -d "$OUT/${v}_$rep" -o a --output-format csv -- "$@" \
      > "$OUT/${v}_$rep.log" 2>&1 || { echo "variant $v failed"; tail -5 "$OUT/${v}_$rep.log"; exit 1; }
  done
done
