#!/bin/bash
# Selected GPU tests (pytest -k expression), then one bench line.
#   gpurun -- bash scripts/gpu_tests_bench.sh "fuse_sum or pow2" [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K=${1:-"fuse_sum"}
shift
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  -k "$K" > gpurun_out/gtb.log 2>&1
rc=$?; tail -30 gpurun_out/gtb.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > gpurun_out/gtb_bench.log 2>&1 \
  || { tail -20 gpurun_out/gtb_bench.log; exit 1; }
grep '^{' gpurun_out/gtb_bench.log | cut -c1-400
