#!/bin/bash
# Final-HEAD evidence in one call: -m gpu suite, default bench line, profiled bench + trace,
# then the PMC HBM traffic of the kernel the default line reports as dominant.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r5i}
bash scripts/archive/gpu_r5_final_a.sh $TAG || exit 1
K=$(grep '^{' gpurun_out/${TAG}_bench_default.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["roofline"]["kernel"])')
echo "dominant: $K"
bash scripts/gpu_pmc.sh ${TAG}_dom "$K" || exit 1
cat gpurun_out/${TAG}_dom_pmc_traffic.json | cut -c1-300
