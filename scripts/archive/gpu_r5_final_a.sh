#!/bin/bash
# Round-5 evidence, part A: the full -m gpu suite, the default bench line (CPU baseline
# included), the profiled bench + rocprofv3 kernel trace / stats + step breakdown.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r5f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_default.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_default.log | cut -c1-300
bash scripts/gpu_bench_prof.sh $TAG || exit 1
