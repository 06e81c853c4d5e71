#!/bin/bash
# Narrow weight gradient: minimum tiles per split 2 (default) vs 1 (twice the workgroups).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 2 1 2 1; do
  VAE2_WGN_MINTPS=$m timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 30 \
    > gpurun_out/r5y_$m.log 2>&1 || { tail -5 gpurun_out/r5y_$m.log; exit 1; }
  echo "== min tps $m"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5y_$m.log
done
for m in 2 1 2 1; do
  VAE2_WGN_MINTPS=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
    > gpurun_out/r5y_bench_$m.log 2>&1 || { tail -20 gpurun_out/r5y_bench_$m.log; exit 1; }
  echo "[bench min tps $m] $(grep '^{' gpurun_out/r5y_bench_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
