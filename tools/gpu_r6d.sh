set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; OUT=gpurun_out/r6d; mkdir -p $OUT
bash tools/ab_builds.sh r6d python3 tools/fbench.py --splats 10000 50000 --iters 400 || exit 1
GSVC_DIAG_LIB=$R/gsvc_amd/lib/alt/hoist/libgsvc_amd_diag.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/rec24 -o a --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 400 --set 24 1 > $OUT/rec24.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $OUT/pmc10k -o p --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 100 > $OUT/pmc10k.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVES -d $OUT/pmc10kb -o p --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 100 > $OUT/pmc10kb.log 2>&1 || exit 1
for d in base_1 hoist_1 base_2 hoist_2 rec24; do echo "== $d"; python3 tools/prof_summary.py --trace $OUT/$d --last 400 2>&1 | grep -E "raster_sum_fwd|frame_project" | head -4; done
python3 - $OUT <<'PY'
import csv, glob, sys, json, collections
for sub in ("pmc10k", "pmc10kb"):
    f = glob.glob(f"{sys.argv[1]}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        for key in ("raster_sum_fwd", "frame_project"):
            if key in r["Kernel_Name"]:
                by[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(sub, json.dumps({k: {c: round(sum(v[-50:]) / len(v[-50:])) for c, v in d.items()} for k, d in by.items()}))
PY
