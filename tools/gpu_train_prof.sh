#!/bin/bash
# Kernel trace + PMC passes of the fused training iteration (tools/tbench.py,
# 1080p / 50k splats by default) on the GPU box, through gpurun.  One
# rocprofv3 run per counter group, each under its own time limit; outputs in
# gpurun_out/$TAG/ (copy the summaries that are judged into profiles/).
#   bash tools/gpu_train_prof.sh TAG [tbench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-trainprof}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 200 python tools/tbench.py --stamps "$@" > $OUT/tbench.jsonl 2> $OUT/tbench.err || { echo "tbench failed"; tail -20 $OUT/tbench.err; exit 1; }
cat $OUT/tbench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o tt --output-format csv -- python3 tools/tbench.py --iters 50 "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py --trace $OUT/trace > $OUT/trace_summary.txt
cut -c1-150 $OUT/trace_summary.txt | head -12
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o p --output-format csv -- python3 tools/tbench.py --iters 20 --warmup 5 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/prof_summary.py --pmc-dirs $OUT/p* > $OUT/pmc_summary.json 2>&1 || true
head -80 $OUT/pmc_summary.json
