set -o pipefail
bash tools/gpu.sh bench_pmc s5 && bash tools/gpu.sh pmc_valu s5 && bash tools/gpu.sh pmc_sq s5
