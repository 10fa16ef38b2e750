#!/bin/bash
# The GPU-box runner (through gpurun): named recipes, every GPU step under its
# own time limit, logs under gpurun_out/$TAG/, stop at the first failure.
#
#   gpurun -- bash tools/gpu.sh RECIPE TAG [args]
#
# Recipes:
#   steps TAG 'name|seconds|cmd' ...   generic: each cmd via bash, log <name>.log
#   tests TAG [pytest args]            the -m gpu suite
#   bench_pmc TAG                      kernel trace + FETCH_SIZE + WRITE_SIZE passes
#                                      (separate runs) of the bench's workloads
#                                      (tools/pmc_workloads.py) -> pmc_traffic.json
#   pmc_valu TAG                       VALU / LDS / SALU / VMEM instruction counts of
#                                      the trained composite and training tile kernel
#   pmc_sq TAG                         SQ busy / wait / LDS-conflict cycles of the same
#   pmc_final TAG                      both, for train50k and render10k -> pmc_valu.json
#   ablate TAG "bits" [tbench args]    training tile kernel diagnostic bits (knob 13)
#                                      on frozen trained-density steps
#   fbench_ab TAG [fbench args]        composite A/B by fbench + kernel trace
#   shared_ranks TAG                   N = 1, 2, 4 bench ranks sharing one GPU (gloo)
#   final TAG                          bench.py (full) + rocprofv3 kernel trace of the bench
#   alpha_ab TAG [KNOB ['V1 V2']]      alpha path A/B (default knob 9: backward DPP vs shuffle sums;
#                                      knob 18 = 100000: forward without lane-group lists),
#                                      interleaved twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
RECIPE=${1:?recipe}
TAG=${2:?tag}
shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp

run() {  # run NAME SECONDS CMD...: one limited step, log, stop on failure
  local name=$1 secs=$2
  shift 2
  echo "== $name ($secs s)"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc in $(( $(date +%s) - t0 )) s"
  tail -n ${TAIL:-4} "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "step $name failed (rc=$rc)"; exit $rc; fi
}

pmc() {  # pmc NAME COUNTERS... -- CMD: one counter pass, killed hard at its limit
  local name=$1
  shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done
  shift
  echo "== pmc $name: ${ctrs[*]}"
  mkdir -p "$(dirname "$OUT/$name.log")"
  timeout -s KILL 200 rocprofv3 --pmc "${ctrs[@]}" -d "$OUT/$name" -o p --output-format csv -- "$@" \
    > "$OUT/$name.log" 2>&1 || { echo "pmc $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
}

case "$RECIPE" in
steps)
  for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    run "$name" "$secs" bash -c "$cmd"
  done ;;
tests)
  run tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread "$@" ;;
bench_pmc)
  for wl in train50k render10k decode8 oppath alpha50k; do
    run "$wl.trace" 200 rocprofv3 --kernel-trace --stats -d "$OUT/$wl/trace" -o t --output-format csv -- python3 tools/pmc_workloads.py $wl
    pmc "$wl/fetch" FETCH_SIZE -- python3 tools/pmc_workloads.py $wl
    pmc "$wl/write" WRITE_SIZE -- python3 tools/pmc_workloads.py $wl
  done
  for key in train_50000 render_50000; do
    python3 tools/prof_summary.py --trace $OUT/train50k/trace --fetch $OUT/train50k/fetch --write $OUT/train50k/write --last 50 --out $OUT/pmc_traffic.json --key $key > $OUT/$key.txt
  done
  python3 tools/prof_summary.py --trace $OUT/render10k/trace --fetch $OUT/render10k/fetch --write $OUT/render10k/write --last 50 --out $OUT/pmc_traffic.json --key render_10000 > $OUT/render_10000.txt
  python3 tools/prof_summary.py --trace $OUT/decode8/trace --fetch $OUT/decode8/fetch --write $OUT/decode8/write --last 50 --out $OUT/pmc_traffic.json --key video_decode > $OUT/video_decode.txt
  python3 tools/prof_summary.py --trace $OUT/oppath/trace --fetch $OUT/oppath/fetch --write $OUT/oppath/write --last 50 --out $OUT/pmc_traffic.json --key op_path > $OUT/op_path.txt
  python3 tools/prof_summary.py --trace $OUT/alpha50k/trace --fetch $OUT/alpha50k/fetch --write $OUT/alpha50k/write --last 50 --out $OUT/pmc_traffic.json --key alpha_50000 > $OUT/alpha_50000.txt
  cat $OUT/pmc_traffic.json ;;
pmc_valu)
  pmc valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES -- python3 tools/pmc_workloads.py train50k
  python3 - "$OUT" <<'PY'
import csv, glob, sys, json, collections
f = glob.glob(f"{sys.argv[1]}/valu/**/*counter_collection.csv", recursive=True)[0]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    for key in ("raster_sum_fwd", "train_tile_band"):
        if key in r["Kernel_Name"]:
            by[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: {c: round(sum(v[-50:]) / len(v[-50:])) for c, v in d.items()} for k, d in by.items()}))
PY
  ;;
pmc_sq)
  # where the tile kernels' cycles go: two SQ passes over the trained workload
  pmc sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 tools/pmc_workloads.py train50k
  pmc sqb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM -- python3 tools/pmc_workloads.py train50k
  python3 - "$OUT" <<'PY'
import csv, glob, sys, json, collections
by = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("sqa", "sqb"):
    f = glob.glob(f"{sys.argv[1]}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        for key in ("raster_sum_fwd", "train_tile_band", "frame_project", "train_splat"):
            if key in r["Kernel_Name"]:
                by[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: {c: round(sum(v[-50:]) / len(v[-50:])) for c, v in d.items()} for k, d in by.items()}, indent=1))
PY
  ;;
pmc_final)
  # the round's instruction counters (VALU / SALU / LDS / VMEM and the SQ wait
  # buckets) of the tile kernels on the bench's workloads; merged locally by
  # tools/pmc_merge.py gpurun_out/TAG > profiles/pmc_valu.json (bench.py reads it)
  for wl in train50k render10k; do
    pmc "$wl/valu" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python3 tools/pmc_workloads.py $wl
    pmc "$wl/sq" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM -- python3 tools/pmc_workloads.py $wl
  done ;;
ablate)
  BITS=${1:-"0 1 2 4 8 16 32 6"}; shift
  for b in $BITS; do
    run "ablate_$b" 120 python tools/tbench.py --warmup 2000 --frozen 300 --knob-after 13=$b "$@"
  done ;;
fbench_ab)
  run fbench 300 python tools/fbench.py "$@"
  run trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr" -o t --output-format csv -- python3 tools/fbench.py "$@" ;;
shared_ranks)
  run n1 300 python bench.py --no-cpu --no-secondary
  for n in 2 4; do
    GSVC_BENCH_SHARED_GPU=1 run n$n 400 python bench.py --gpus $n --backend gloo --no-cpu
  done ;;
final)
  # the round's bench line (with the CPU baselines) and the kernel trace of the
  # same workload (the bench without its CPU legs), for profiles/rNN/final
  run bench 900 python bench.py
  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o b --output-format csv -- python3 bench.py --no-cpu ;;
alpha_ab)
  KN=${1:-9}; VALS=${2:-"0 1"}
  for rep in 1 2; do
    for k in $VALS; do
      run "k${k}_$rep" 200 rocprofv3 --kernel-trace --stats -d "$OUT/k${k}_$rep" -o a --output-format csv -- python3 tools/alphabench.py --splats 50000 --calls 100 --knob $KN=$k
    done
  done ;;
*)
  echo "unknown recipe $RECIPE"; exit 2 ;;
esac
