set -o pipefail
bash tools/gpu.sh steps r6b \
 'ids10k|300|python -u tools/fbench.py --splats 10000 --iters 200 --id-stamps gpurun_out/r6b/ids10k.npz' \
 'ids50k|300|python -u tools/fbench.py --splats 50000 --trained 2000 --iters 200 --id-stamps gpurun_out/r6b/ids50k.npz' \
 'tr10k|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6b/tr10k -o t --output-format csv -- python3 tools/fbench.py --splats 10000 --iters 200' \
 'tr50k|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6b/tr50k -o t --output-format csv -- python3 tools/fbench.py --splats 50000 --trained 2000 --iters 200'
for d in tr10k tr50k; do python3 tools/prof_summary.py --trace gpurun_out/r6b/$d --last 200 > gpurun_out/r6b/$d.txt 2>&1; head -6 gpurun_out/r6b/$d.txt; done
