#!/bin/bash
# Selected GPU tests (no -x) then conv_bench A/B over vae2_conv2d_set_algo values.
#   gpurun -- bash scripts/gpu_tb.sh "<pytest -k expression>" "<conv_bench --only idx>" "<algos>"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests -m gpu \
    -k "$1" > gpurun_out/gt2.log 2>&1
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gt2.log | tail -40
fi
if [ -n "$2" ]; then
  timeout -k 10 300 python vae-2_amd/tools/conv_bench.py --only $2 --iters 30 --algo ${3:-0} \
    2>&1 | grep -v "amdgpu.ids" | tee gpurun_out/cb.log || exit 1
fi
