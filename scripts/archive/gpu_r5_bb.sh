#!/bin/bash
# World-1 RCCL tests (incl. graph capture) three times in one process each, after the
# capture drain / event-cache change; then the graph and dist suites.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 280 python -u -m pytest -x -q -s --timeout 250 --timeout-method thread tests/test_dist_rccl_gpu.py \
    > gpurun_out/r5bb_$i.log 2>&1
  rc=$?; echo "run $i rc=$rc"; grep -E "passed|failed|rccl graph worker\] (captured|replayed)|hipError" gpurun_out/r5bb_$i.log | head -5
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_graph_gpu.py tests/test_dist_gpu.py \
  > gpurun_out/r5bb_g.log 2>&1; rc=$?; echo "graph/dist rc=$rc"; tail -1 gpurun_out/r5bb_g.log
