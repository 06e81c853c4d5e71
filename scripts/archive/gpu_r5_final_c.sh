#!/bin/bash
# Default bench line, then the PMC HBM traffic of whatever kernel it reports as dominant.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r5h}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_default.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_default.log | cut -c1-200
K=$(grep '^{' gpurun_out/${TAG}_bench_default.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["roofline"]["kernel"])')
echo "dominant: $K"
bash scripts/gpu_pmc.sh ${TAG}_dom "$K" || exit 1
cat gpurun_out/${TAG}_dom_pmc_traffic.json | cut -c1-300
