#!/bin/bash
# SSIM parity tests, timing and a kernel trace (through gpurun).
set -o pipefail
mkdir -p gpurun_out/ss
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ssim.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ssim.log 2>&1 || { tail -30 gpurun_out/ssim.log; exit 1; }
tail -1 gpurun_out/ssim.log
timeout -k 10 300 python tools/ssimbench.py "$@" > gpurun_out/ss/ssimbench.jsonl 2> gpurun_out/ss/err.log || { tail gpurun_out/ss/err.log; exit 1; }
cat gpurun_out/ss/ssimbench.jsonl
rm -rf gpurun_out/ss/tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ss/tr -o s --output-format csv -- python3 tools/ssimbench.py --only-hip --iters 20 > gpurun_out/ss/tr.log 2>&1 || { tail gpurun_out/ss/tr.log; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/ss/tr ssim
