#!/bin/bash
# The world-1 RCCL graph-capture test alone, verbose, with progress markers.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 280 python -u -m pytest -x -v -s --timeout 260 --timeout-method thread \
  tests/test_dist_rccl_gpu.py 2>&1 | tee gpurun_out/r5w.log | grep -v amdgpu.ids
