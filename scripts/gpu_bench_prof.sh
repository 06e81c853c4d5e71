#!/bin/bash
# bench.py (live per-family profile) and a rocprofv3 kernel-trace of the same command.
#   gpurun --timeout 900 -- bash scripts/gpu_bench_prof.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-bp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline --profile-json gpurun_out/${TAG}_profile.json \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-600
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o run -- \
  python bench.py --no-cpu-baseline --profile-json gpurun_out/${TAG}_profile_rp.json \
  > gpurun_out/${TAG}_bench_rp.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_rp.log; exit 1; }
CSV=$(find gpurun_out/${TAG}_prof -name '*kernel_trace.csv' | head -1)
# the 8 last graph-replayed timed steps (bench.py's 3 eager roofline steps come after them)
python vae-2_amd/tools/trace_steps.py "$CSV" --steps 8 --skip 3 --json gpurun_out/${TAG}_steps.json \
  > gpurun_out/${TAG}_steps.txt 2>&1
head -40 gpurun_out/${TAG}_steps.txt
