set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; OUT=gpurun_out/r6k; mkdir -p $OUT
bash tools/gpu.sh steps r6k \
 'tests|600|python -u -m pytest tests/test_train_fused.py tests/test_train_trajectory.py tests/test_trained_state.py tests/test_deterministic.py tests/test_carried_bins.py -m gpu -x -q --timeout 120 --timeout-method thread' \
 'ab_p1|200|python -u tools/tbench.py --warmup 2000 --frozen 300' \
 'ab_s1|200|python -u tools/tbench.py --warmup 2000 --frozen 300 --knob-after 13=512' \
 'ab_p2|200|python -u tools/tbench.py --warmup 2000 --frozen 300' \
 'ab_s2|200|python -u tools/tbench.py --warmup 2000 --frozen 300 --knob-after 13=512' \
 'bench|600|python -u bench.py --no-cpu --no-secondary'
