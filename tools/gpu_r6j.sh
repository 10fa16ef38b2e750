set -o pipefail
bash tools/gpu.sh steps r6j \
 'tests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
 'smoke|300|python -c "import __graft_entry__ as g; g.smoke()"' \
 'bench|600|python -u bench.py --no-cpu' \
 'prof|600|rocprofv3 --kernel-trace --stats -d gpurun_out/r6j/prof -o b --output-format csv -- python3 bench.py --no-cpu --no-secondary'
