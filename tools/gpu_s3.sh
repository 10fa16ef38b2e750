set -o pipefail
mkdir -p gpurun_out/s3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/s3/prof_skel -o skel -- ./tools/micro/bin/composite_skeleton > gpurun_out/s3/skeleton_prof.log 2>&1 \
&& timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_torch_ops.py tests/test_store_hazard.py tests/test_trained_state.py tests/test_capture.py -m gpu > gpurun_out/s3/gpu_tests.log 2>&1 \
&& timeout -k 10 300 python -u bench.py > gpurun_out/s3/bench.log 2>&1
