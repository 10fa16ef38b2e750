set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; OUT=gpurun_out/r6e; mkdir -p $OUT
bash tools/gpu.sh steps r6e \
 'tests|600|python -u -m pytest tests/test_id_slabs.py tests/test_gpu_parity.py tests/test_store_hazard.py tests/test_trained_state.py tests/test_video.py -m gpu -x -q --timeout 120 --timeout-method thread' \
 'ab1|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6e/ab1 -o a --output-format csv -- python3 tools/fbench.py --splats 10000 50000 --iters 400 --knob 38 1' \
 'ab2|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6e/ab2 -o a --output-format csv -- python3 tools/fbench.py --splats 10000 50000 --iters 400 --knob 38 1' \
 'tr50k|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6e/tr50k -o a --output-format csv -- python3 tools/fbench.py --splats 50000 --trained 2000 --iters 400 --knob 38 1' \
 'ids10k|300|python -u tools/fbench.py --splats 10000 --iters 200 --id-stamps gpurun_out/r6e/ids10k.npz'
for d in ab1 ab2 tr50k; do echo "== $d"; python3 tools/trace_runs.py $OUT/$d raster_render_ids; python3 tools/trace_runs.py $OUT/$d raster_sum_fwd; done
