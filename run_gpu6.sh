#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r6_prof.log 2>&1
echo rc=$?
