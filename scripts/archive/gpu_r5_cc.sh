#!/bin/bash
# The default bench line alone (CPU baseline, roofline with the committed PMC traffic).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r5cc_bench_default.log 2>&1 || { tail -20 gpurun_out/r5cc_bench_default.log; exit 1; }
grep '^{' gpurun_out/r5cc_bench_default.log | cut -c1-300
