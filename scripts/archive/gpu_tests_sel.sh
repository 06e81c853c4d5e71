#!/bin/bash
# Selected GPU tests (pytest -k expression) + optional conv microbench shapes.
#   gpurun -- bash scripts/gpu_tests_sel.sh "multi_bn" "3 4"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K=${1:-"multi_bn"}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  -k "$K" > gpurun_out/gt1.log 2>&1
rc=$?; tail -25 gpurun_out/gt1.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$2" ]; then
  timeout -k 10 300 python vae-2_amd/tools/conv_bench.py --only $2 --iters 20 --algo 0
fi
