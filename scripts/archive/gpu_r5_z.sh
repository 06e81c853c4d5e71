#!/bin/bash
# Per-module bf16-operand gradient checks (stage modules, heads).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread \
  tests/test_bf16_gpu.py -k "per_module or heads_gradients" > gpurun_out/r5z.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "gradients, min cosine|PASS|FAIL|assert|Error" gpurun_out/r5z.log | head -20
