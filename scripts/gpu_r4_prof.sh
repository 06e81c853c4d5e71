#!/bin/bash
# Round-4 profiling call: igemm launch-shape A/B over every ELBO conv shape, SQ stall
# counters of the narrow conv kernels, then the profiled bench + rocprofv3 kernel trace.
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_prof.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-p4}
mkdir -p gpurun_out
export TMPDIR=/tmp
for tune in "" "0=512" "0=1024" "1=1" "2=1" "3=1"; do
  timeout -k 10 240 python vae-2_amd/tools/conv_bench.py --all --iters 20 ${tune:+--tune $tune} \
    > gpurun_out/${TAG}_cb_${tune:-default}.log 2>&1 || { tail -5 gpurun_out/${TAG}_cb_${tune:-default}.log; exit 1; }
  echo "== tune '${tune}'"; grep "weighted" gpurun_out/${TAG}_cb_${tune:-default}.log
done
bash scripts/gpu_narrow_pmc.sh ${TAG}_n "2 3 4 5 9" || exit 1
bash scripts/gpu_bench_prof.sh ${TAG} || exit 1
