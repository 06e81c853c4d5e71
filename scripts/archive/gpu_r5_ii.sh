#!/bin/bash
# bf16-operand and 256x512 lines at the final round-5 HEAD.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r5k
mkdir -p gpurun_out
export TMPDIR=/tmp
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
