#!/bin/bash
# Full -m gpu suite, then one bench line (no CPU baseline).
#   gpurun --timeout 1100 -- bash scripts/gpu_full.sh [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/full_tests.log 2>&1
rc=$?; tail -15 gpurun_out/full_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/head_bench.log 2>&1 \
  || { tail -20 gpurun_out/head_bench.log; exit 1; }
grep '^{' gpurun_out/head_bench.log | cut -c1-500
