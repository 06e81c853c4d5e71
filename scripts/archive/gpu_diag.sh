#!/bin/bash
# gpurun -- bash scripts/gpu_diag.sh <python script> [args]: one diagnostic script, time-limited.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u "$@" > gpurun_out/diag.log 2>&1
rc=$?; tail -60 gpurun_out/diag.log; exit $rc
