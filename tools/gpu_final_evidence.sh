set -o pipefail
# The round's closing evidence on ONE box (the library as committed): the SQ
# instruction / wait counters of the bench's tile kernels (tools/gpu.sh
# pmc_final, merged on the box into pmc_valu.json), then bench.py and its own
# kernel trace (tools/gpu.sh final), the trace summaries, and the raw CSVs
# over 2 MB deleted so gpurun_out/ stays under the 64 MiB it copies back.
T=${1:-final}
O=gpurun_out/$T
bash tools/gpu.sh pmc_final $T && \
python3 tools/pmc_merge.py $O > $O/pmc_valu.json && \
bash tools/gpu.sh final $T && \
python3 tools/prof_summary.py --trace $O/prof > $O/bench_kernel_trace_summary.txt && \
python3 tools/trace_runs.py $O/prof raster_render_ids > $O/bench_trace_render_runs.txt && \
find $O -name '*.csv' -size +2M -delete
