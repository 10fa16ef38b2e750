#!/bin/bash
# Projection insertion A/B (knob 2 = 4: one 32-bit slot atomic per tile instead
# of paired 64-bit ones): parity tests, fbench and per-pass projection traces.
set -o pipefail
mkdir -p gpurun_out/pa
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync_free.py tests/test_train_fused.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pa/t.log 2>&1 || { tail -30 gpurun_out/pa/t.log; exit 1; }
tail -1 gpurun_out/pa/t.log
timeout -k 10 200 python tools/fbench.py --splats 10000 50000 --knob 2 4 || exit 1
timeout -k 10 200 python tools/fbench.py --splats 50000 --chol-scale 8 --knob 2 4 || exit 1
rm -rf gpurun_out/pa/tr
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pa/tr -o t --output-format csv -- python3 tools/fbench.py --splats 50000 --chol-scale 8 --iters 100 --knob 2 4 > gpurun_out/pa/tr.log 2>&1 || { tail gpurun_out/pa/tr.log; exit 1; }
python3 tools/split_trace.py gpurun_out/pa/tr frame_project 401
