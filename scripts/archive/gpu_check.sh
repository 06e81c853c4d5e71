#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench.  Usage (from this container):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_check.sh TAG
# Every GPU step runs under its own time limit; the script stops at the first
# abort / fault / timeout so nothing else touches a GPU in a bad state.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-chk}
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local t=$1; local log=$2; shift 2
  echo "== $* (> $log)"
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/${TAG}_$log"
  echo "== rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step 600 tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 500 bench.log python bench.py
grep '^{' "gpurun_out/${TAG}_bench.log" | cut -c1-400
