#!/bin/bash
# Narrow 3x3 weight gradient with the chunk loop software-pipelined: tests + conv_bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_narrow_gpu.py \
  > gpurun_out/r5r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5r_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5r_tests.log | head -20; exit $rc; }
for t in 7=0 7=1; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 20 --tune $t \
    > gpurun_out/r5r_conv_$t.log 2>&1 || { tail -5 gpurun_out/r5r_conv_$t.log; exit 1; }
  echo "== conv tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5r_conv_$t.log
done
