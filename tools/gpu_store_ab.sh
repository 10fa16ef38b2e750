#!/bin/bash
# A/B of store cache policies (knob 6: projection records, knob 7: composite
# planes) by fbench µs/frame and per-pass kernel-trace durations (through gpurun).
set -o pipefail
mkdir -p gpurun_out/st
export TMPDIR=/tmp
timeout -k 10 300 python tools/fbench.py --splats 10000 50000 --knob 6 1 --knob 7 1 --knob 7 4 > gpurun_out/st/fbench.jsonl 2>gpurun_out/st/fbench.err || { tail gpurun_out/st/fbench.err; exit 1; }
cat gpurun_out/st/fbench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/st/tr -o t --output-format csv -- python3 tools/fbench.py --splats 10000 --knob 6 1 --knob 7 1 --knob 7 4 > gpurun_out/st/tr.log 2>&1 || { tail gpurun_out/st/tr.log; exit 1; }
python3 tools/split_trace.py gpurun_out/st/tr raster_sum_fwd 801
python3 tools/split_trace.py gpurun_out/st/tr frame_project 801
