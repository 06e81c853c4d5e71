#!/bin/bash
# Direct 3x3 with 16-channel N blocks for layers short of workgroups (key 13): the 72 / 144-
# channel shapes, conv tests with it on, step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 13=0 13=1 13=0 13=1; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 5 6 --iters 30 --tune $t \
    > gpurun_out/r5ee_$t.log 2>&1 || { tail -5 gpurun_out/r5ee_$t.log; exit 1; }
  echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5ee_$t.log
done
for t in 13=0 13=1 13=0 13=1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5ee_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5ee_bench_$t.log; exit 1; }
  echo "[bench $t] $(grep '^{' gpurun_out/r5ee_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
