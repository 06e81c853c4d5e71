#!/bin/bash
# bench.py under different values of one environment variable, in turn (A/B on one box).
#   gpurun -- bash scripts/gpu_envab.sh VAR "v1 v2 v3"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VAR=$1; VALS=$2
i=0
for v in $VALS $VALS; do
  i=$((i+1))
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
    > gpurun_out/envab_$i.log 2>&1 || { tail -20 gpurun_out/envab_$i.log; exit 1; }
  echo "[$VAR=$v] $(grep '^{' gpurun_out/envab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
