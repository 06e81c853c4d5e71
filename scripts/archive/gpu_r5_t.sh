#!/bin/bash
# Stride-2 convs (gather kernel): row-tile shrink (key 0) and VALU remainder (key 6) sweep.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 0=0 0=512 0=1024 0=2048 6=1 6=1,0=1024; do
  timeout -k 10 150 python vae-2_amd/tools/conv_bench.py --all --only 6 8 9 15 16 17 18 24 25 26 --iters 20 --tune $t \
    > gpurun_out/r5t_$t.log 2>&1 || { tail -5 gpurun_out/r5t_$t.log; exit 1; }
  echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5t_$t.log
done
