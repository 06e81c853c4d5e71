#!/bin/bash
# Selected GPU tests (pytest -k), the head microbenchmark, then bench A/B runs.
#   gpurun -- bash scripts/gpu_quick.sh "bn or multi" "--graph on" "--graph off"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K=$1; shift
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  -k "$K" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/quick_tests.log | head -20; exit $rc; }
timeout -k 10 120 python vae-2_amd/tools/head_bench.py > gpurun_out/quick_head.log 2>&1 \
  && grep -E "upsum|adjoint|head_out" gpurun_out/quick_head.log
bash scripts/gpu_ab.sh "$@"
