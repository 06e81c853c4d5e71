#!/bin/bash
# Kernel-trace profile of the bench + per-step breakdown.  Usage:
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_profile.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o run -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_prof.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench_prof.log; exit $rc; }
grep '^{' gpurun_out/${TAG}_bench_prof.log | cut -c1-200
CSV=$(find gpurun_out/${TAG}_prof -name '*kernel_trace.csv' | head -1)
python vae-2_amd/tools/trace_steps.py "$CSV" --steps 10 > gpurun_out/${TAG}_steps.txt 2>&1
cat gpurun_out/${TAG}_steps.txt | head -60
