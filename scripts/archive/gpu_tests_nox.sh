#!/bin/bash
# Selected GPU tests without -x (every selected test runs; -s shows their printed tables).
#   gpurun -- bash scripts/gpu_tests_nox.sh "<pytest -k expression>"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests -m gpu \
  -k "$1" > gpurun_out/gt2.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gt2.log | tail -30
exit $rc
