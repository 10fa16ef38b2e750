set -o pipefail
# the round's bench evidence on ONE box: the PMC traffic and trace passes of the
# bench's workloads (tools/gpu.sh bench_pmc), installed as profiles/pmc_traffic.json
# in this box's copy so bench.py's trace fields come from the same box, then the
# full bench line and its own kernel trace (tools/gpu.sh final)
T=${1:-r6fin2}
bash tools/gpu.sh bench_pmc $T && cp gpurun_out/$T/pmc_traffic.json profiles/pmc_traffic.json && \
bash tools/gpu.sh final $T
