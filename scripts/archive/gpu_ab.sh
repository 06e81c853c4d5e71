#!/bin/bash
# A/B of one bench.py switch on the same box: bench A, bench B, bench A again.
#   gpurun -- bash scripts/gpu_ab.sh "--conv-grouping on" "--conv-grouping off"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$1; B=$2; shift 2
i=0
for args in "$A" "$B" "$A" "$B"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 $args "$@" \
    > gpurun_out/ab_$i.log 2>&1 || { tail -20 gpurun_out/ab_$i.log; exit 1; }
  echo "[$args] $(grep '^{' gpurun_out/ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
