set -o pipefail
mkdir -p gpurun_out/s2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/micro/bin/composite_skeleton > gpurun_out/s2/skeleton.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/prof_skel -o skel -- ./tools/micro/bin/composite_skeleton > gpurun_out/s2/skeleton_prof.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/s2/gpu_tests.log 2>&1 \
&& timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/hwc_plain -o p -- python3 tools/hwc_store_ab.py > gpurun_out/s2/hwc_plain.log 2>&1 \
&& GSVC_DIAG_LIB=gsvc_amd/lib/repro/libgsvc_amd_r5hwc_nop.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/hwc_wt -o p -- python3 tools/hwc_store_ab.py > gpurun_out/s2/hwc_wt.log 2>&1 \
&& timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/hwc_plain2 -o p -- python3 tools/hwc_store_ab.py > gpurun_out/s2/hwc_plain2.log 2>&1
