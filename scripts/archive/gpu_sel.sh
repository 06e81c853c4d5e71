#!/bin/bash
# Selected GPU test files / -k expression (no bench).
#   gpurun -- bash scripts/gpu_sel.sh "tests/test_clips_gpu.py tests/test_metrics_gpu.py" [-k EXPR]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FILES=$1
shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $FILES -m gpu "$@" \
  > gpurun_out/sel.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/sel.log | tail -40; tail -3 gpurun_out/sel.log
exit $rc
