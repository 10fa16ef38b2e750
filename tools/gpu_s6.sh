set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/s6; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $OUT/gpu_tests.log; exit 1; }
for b in 0 4 8 16 256; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES -d $OUT/lds_$b -o p --output-format csv -- python3 tools/tbench.py --warmup 2000 --frozen 300 --knob-after 13=$b > $OUT/lds_$b.log 2>&1 || { echo pmc $b failed; tail -5 $OUT/lds_$b.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, json, collections
for b in (0, 4, 8, 16, 256):
    f = glob.glob(f"{sys.argv[1]}/lds_{b}/**/*counter_collection.csv", recursive=True)[0]
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "train_tile_band" in r["Kernel_Name"]:
            by[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(b, json.dumps({c: round(sum(v[-50:]) / len(v[-50:])) for c, v in by.items()}))
PY
