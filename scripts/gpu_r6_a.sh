#!/bin/bash
# Round 6: SyncBN failure semantics, capture drain, key-6 default form vs fp64.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_abi.py tests/test_syncbn_ipc_gpu.py tests/test_dist_rccl_gpu.py \
  "tests/test_model_gpu.py::test_w18_gather_remainder_form_gradients_vs_fp64" \
  tests/test_dist_gpu.py -s > gpurun_out/r6_a.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|error|PASS|FAIL|median|exact|captured|drain" gpurun_out/r6_a.log | tail -40
exit $rc
