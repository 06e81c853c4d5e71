#!/bin/bash
# Round-5 evidence, part B: PMC HBM traffic of the dominant kernel, bf16-operand and
# 256x512 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r5f}
KERNEL=${2:-"wgrad3n_kernel<9, 2, 4, 1, false>"}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh ${TAG}_dom "$KERNEL" || exit 1
cat gpurun_out/${TAG}_dom_pmc_traffic.json | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu-baseline --dtype bf16 \
  --profile-json gpurun_out/${TAG}_profile_bf16.json > gpurun_out/${TAG}_bench_bf16.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_bf16.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_bf16.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --height 256 --width 512 --batch 2 \
  > gpurun_out/${TAG}_bench_256x512.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_256x512.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_256x512.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --dtype bf16 --height 256 --width 512 --batch 2 \
  > gpurun_out/${TAG}_bench_bf16_256x512.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_bf16_256x512.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_bf16_256x512.log | cut -c1-200
