set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g1/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/g1/gpu_tests.log; exit 1; }
tail -2 gpurun_out/g1/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1/smoke.log 2>&1 || { tail -20 gpurun_out/g1/smoke.log; exit 1; }
tail -1 gpurun_out/g1/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err || { tail -20 gpurun_out/g1/bench.err; exit 1; }
cut -c1-600 gpurun_out/g1/bench.json
