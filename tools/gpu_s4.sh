set -o pipefail
mkdir -p gpurun_out/s4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/prof_skel -o skel -- ./tools/micro/bin/composite_skeleton > gpurun_out/s4/skeleton_prof.log 2>&1 \
&& timeout -k 10 300 python -u tools/fbench.py --splats 10000 --stamps --iters 200 > gpurun_out/s4/stamps10k.log 2>&1 \
&& timeout -k 10 300 python -u tools/fbench.py --splats 50000 --trained 2000 --stamps --iters 200 > gpurun_out/s4/stamps50k.log 2>&1
