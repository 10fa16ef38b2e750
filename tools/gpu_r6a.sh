set -o pipefail
bash tools/gpu.sh steps r6a \
 'tests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
 'stamps10k|300|python -u tools/fbench.py --splats 10000 --stamps --iters 200' \
 'stamps50k|300|python -u tools/fbench.py --splats 50000 --trained 2000 --stamps --iters 200' \
 'bench|600|python -u bench.py --no-cpu' \
 'prof|600|rocprofv3 --kernel-trace --stats -d gpurun_out/r6a/prof -o b --output-format csv -- python3 bench.py --no-cpu --no-secondary'
