#!/bin/bash
# Final check of the committed tree: full -m gpu suite and smoke().
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/r5ff_tests.log 2>&1 || { tail -30 gpurun_out/r5ff_tests.log; exit 1; }
tail -1 gpurun_out/r5ff_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ff_smoke.log 2>&1 || { tail -20 gpurun_out/r5ff_smoke.log; exit 1; }
tail -3 gpurun_out/r5ff_smoke.log
