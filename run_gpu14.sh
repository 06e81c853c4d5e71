#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r14 -o run -- python bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 2 > gpurun_out/r14_prof.log 2>&1
grep '^{' gpurun_out/r14_prof.log | cut -c1-200
ls -R gpurun_out/prof_r14 | head
