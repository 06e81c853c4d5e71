#!/bin/bash
# Round 6: bf16 gradient tests with the in-test calibration
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_bf16_gpu.py \
  > gpurun_out/r6_h_bf16.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|gradients, min cosine|Error" gpurun_out/r6_h_bf16.log | tail -30
exit $rc
