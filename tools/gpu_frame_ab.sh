#!/bin/bash
# Frame-path parity tests, then render / training timings and a per-pass
# kernel-trace split of the 10k render (through gpurun).
set -o pipefail
mkdir -p gpurun_out/fa
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync_free.py tests/test_train_fused.py tests/test_frame_train.py tests/test_video.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fa/t.log 2>&1 || { tail -30 gpurun_out/fa/t.log; exit 1; }
tail -1 gpurun_out/fa/t.log
timeout -k 10 200 python tools/fbench.py --splats 10000 50000 100000 --proj-stamps "$@" || exit 1
timeout -k 10 200 python tools/tbench.py || exit 1
rm -rf gpurun_out/fa/tr
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fa/tr -o t --output-format csv -- python3 tools/fbench.py --splats 10000 "$@" > gpurun_out/fa/tr.log 2>&1 || { tail gpurun_out/fa/tr.log; exit 1; }
python3 tools/split_trace.py gpurun_out/fa/tr raster_sum_fwd 801
python3 tools/split_trace.py gpurun_out/fa/tr frame_project 801
