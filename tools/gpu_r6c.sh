set -o pipefail
bash tools/gpu.sh steps r6c \
 'tests|600|python -u -m pytest tests/test_carried_bins.py tests/test_train_fused.py tests/test_adan.py tests/test_train_trajectory.py tests/test_trained_state.py tests/test_deterministic.py -m gpu -x -q --timeout 120 --timeout-method thread' \
 'splat_e1|200|python -u tools/tbench.py --channels --knob 34=0' \
 'splat_s1|200|python -u tools/tbench.py --channels --knob 34=2' \
 'splat_o1|200|python -u tools/tbench.py --channels --knob 34=1' \
 'splat_e2|200|python -u tools/tbench.py --channels --knob 34=0' \
 'splat_s2|200|python -u tools/tbench.py --channels --knob 34=2' \
 'ids10k|300|python -u tools/fbench.py --splats 10000 --iters 200 --id-stamps gpurun_out/r6c/ids10k.npz' \
 'ids50k|300|python -u tools/fbench.py --splats 50000 --trained 2000 --iters 200 --id-stamps gpurun_out/r6c/ids50k.npz' \
 'tr10k|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6c/tr10k -o t --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 200' \
 'bench|600|python -u bench.py --no-cpu --no-secondary'
python3 tools/prof_summary.py --trace gpurun_out/r6c/tr10k --last 200 > gpurun_out/r6c/tr10k.txt 2>&1; head -5 gpurun_out/r6c/tr10k.txt
