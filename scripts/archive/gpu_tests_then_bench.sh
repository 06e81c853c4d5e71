#!/bin/bash
# Full -m gpu suite (or a -k selection), then one default bench line.
#   gpurun --timeout 1200 -- bash scripts/gpu_tests_then_bench.sh TAG ["-k expr"] [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-tb}; K=${2:-}; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest --maxfail=4 -v --timeout 420 --timeout-method thread tests -m gpu \
    -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest --maxfail=4 -v --timeout 420 --timeout-method thread tests -m gpu \
    > gpurun_out/${TAG}_tests.log 2>&1
fi
rc=$?; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-600
