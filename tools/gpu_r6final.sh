set -o pipefail
# the round's evidence for the committed library, part 1: GPU suite + smoke,
# PMC traffic and instruction passes (merged into profiles/ locally); part 2 is
# `bash tools/gpu.sh final TAG` (bench.py reads the refreshed profiles/)
bash tools/gpu.sh tests ${1:-r6fin} && \
bash tools/gpu.sh steps ${1:-r6fin} 'smoke|300|python -c "import __graft_entry__ as g; g.smoke()"' && \
bash tools/gpu.sh bench_pmc ${1:-r6fin} && \
bash tools/gpu.sh pmc_final ${1:-r6fin}
