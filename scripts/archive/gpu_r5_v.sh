#!/bin/bash
# Narrow weight gradient: per-tile staging (key 7 = 1) vs register prefetch of the next tile
# (7 = 2) on the 18 / 36 / 72-channel shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 7=1 7=2 7=1 7=2; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 30 --tune $t \
    > gpurun_out/r5v_$t.log 2>&1 || { tail -5 gpurun_out/r5v_$t.log; exit 1; }
  echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5v_$t.log
done
