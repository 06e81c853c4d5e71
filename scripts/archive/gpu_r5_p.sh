#!/bin/bash
# 72 / 144-channel 3x3 layers: direct vs gather kernels (+ gather row-tile shrink, key 0).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 5 6 --iters 20 --algo 0 1 \
  > gpurun_out/r5p_a.log 2>&1 || { tail -5 gpurun_out/r5p_a.log; exit 1; }
grep -E "^==|^[0-9]+x[0-9]+" gpurun_out/r5p_a.log
for t in 0=512 0=1024 0=2048; do
timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 5 6 --iters 20 --algo 1 --tune $t \
  > gpurun_out/r5p_$t.log 2>&1 || { tail -5 gpurun_out/r5p_$t.log; exit 1; }
echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5p_$t.log
done
