#!/bin/bash
# Round-4 profiling call: the profiled bench + rocprofv3 kernel trace + step breakdown,
# then SQ stall counters of the narrow conv kernels (conv_bench shapes).
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_prof.sh TAG "3 4 9"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-p4}
IDX=${2:-"3 4 9"}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_bench_prof.sh ${TAG} || exit 1
bash scripts/gpu_narrow_pmc.sh ${TAG}_n "$IDX" || exit 1
