#!/bin/bash
# Full-flush event ordering for the anchor's own-stream flush: dist / graph / model tests + bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_dist_rccl_gpu.py \
  tests/test_dist_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py tests/test_lazy_bn_gpu.py > gpurun_out/r5x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5x_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5x_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 > gpurun_out/r5x_bench.log 2>&1 || { tail -20 gpurun_out/r5x_bench.log; exit 1; }
grep '^{' gpurun_out/r5x_bench.log | cut -c1-200
