#!/bin/bash
# Training-step A/B of vae2_heads_set_algo settings (bench.py --heads-algo), interleaved.
#   gpurun --timeout 900 -- bash scripts/gpu_r4_hab.sh TAG "0 64 128 192"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-hab}
ALGOS=${2:-"0 64 128 192"}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for rep in 1 2; do
  for v in $ALGOS; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 --heads-algo $v \
      > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    echo "[$v] $(grep '^{' gpurun_out/${TAG}_ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
