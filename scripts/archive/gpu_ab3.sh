#!/bin/bash
# bench.py under several argument sets, twice each (interleaved), on one box.
#   gpurun -- bash scripts/gpu_ab3.sh "--bn-apply-iters 1" "--bn-apply-iters 2" "--bn-apply-iters 4"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for args in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 $args > gpurun_out/ab3_$i.log 2>&1 \
      || { tail -20 gpurun_out/ab3_$i.log; exit 1; }
    echo "[$args] $(grep '^{' gpurun_out/ab3_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); f=d.get("families",{}).get("batchnorm",{}); print(d["value"], d["ms_per_step"], "bn_ms", f.get("ms_per_step"))')"
  done
done
