#!/bin/bash
# Gather GEMM VALU remainder for 18 output channels only (key 6 = 2) vs off: all conv shapes, step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 6=0 6=2; do
  timeout -k 10 200 python vae-2_amd/tools/conv_bench.py --all --iters 20 --tune $t > gpurun_out/r5gg_$t.log 2>&1 || { tail -5 gpurun_out/r5gg_$t.log; exit 1; }
  echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5gg_$t.log | grep -E "\->18 |18->"
done
for t in 6=0 6=2 6=0 6=2 6=0 6=2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5gg_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5gg_bench_$t.log; exit 1; }
  echo "[bench $t] $(grep '^{' gpurun_out/r5gg_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
