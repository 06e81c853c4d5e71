#!/bin/bash
# Round-end evidence in one call: full -m gpu suite, the default bench line (with the CPU
# baseline), the profiled bench + rocprofv3 kernel trace and step breakdown, the bf16
# line, and the dominant kernel's PMC HBM traffic.
#   gpurun --timeout 1200 -- bash scripts/gpu_final.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_default.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_default.log | cut -c1-300
bash scripts/gpu_bench_prof.sh $TAG || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --dtype bf16 \
  --profile-json gpurun_out/${TAG}_profile_bf16.json > gpurun_out/${TAG}_bench_bf16.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_bf16.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_bf16.log | cut -c1-200
bash scripts/gpu_pmc.sh ${TAG}_bnapply bn_bwd_apply_multi_kernel
timeout -k 10 300 python bench.py --no-cpu-baseline --dtype bf16 --height 256 --width 512 --batch 2 \
  > gpurun_out/${TAG}_bench_bf16_256x512.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_bf16_256x512.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_bf16_256x512.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --height 256 --width 512 --batch 2 \
  > gpurun_out/${TAG}_bench_256x512.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_256x512.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_256x512.log | cut -c1-200
