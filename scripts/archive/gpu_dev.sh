#!/bin/bash
# Development loop on the GPU box: selected tests first, then all GPU tests and the
# bench.  Usage: gpurun --timeout 1200 -- bash scripts/gpu_dev.sh TAG "tests/test_x.py ..."
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-dev}
FIRST=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local t=$1; local log=$2; shift 2
  echo "== $* (> $log)"
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$log" 2>&1
  local rc=$?
  tail -15 "gpurun_out/${TAG}_$log"
  echo "== rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -n "$FIRST" ]; then
  step 400 first.log python -u -m pytest $FIRST -x -q --timeout 200 --timeout-method thread
fi
step 600 tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 500 bench.log python bench.py --no-cpu-baseline
grep '^{' "gpurun_out/${TAG}_bench.log" | cut -c1-300
