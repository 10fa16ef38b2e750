#!/bin/bash
# Full GPU suite + bench A/B of the grouped forward (knob 15) + frozen tile timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/s3e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for k in 0 1 0; do
timeout -k 10 300 python bench.py --no-cpu --knob 15=$k > $OUT/bench_k$k.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "
import json,sys;d=json.load(open('$OUT/bench_k$k.json'))
print('knob15=$k', d['value'], d['kernels']['train_tile']['avg_kernel_us'], 'render', d['render']['frames_per_s'], d['render']['roofline']['avg_kernel_us'], '10k', d['render_10k']['frames_per_s'], d['render_10k']['roofline']['avg_kernel_us'], 'gop', d['video_decode']['frames_per_s'])"
done
for k in 0 0; do
timeout -k 10 120 python tools/tbench.py --warmup 2000 --frozen 300 --knob-after 13=$k >> $OUT/frozen.jsonl 2>> $OUT/tb.err || { tail -20 $OUT/tb.err; exit 1; }
tail -1 $OUT/frozen.jsonl | cut -c1-300
done
