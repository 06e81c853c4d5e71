#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 600 python -m pytest tests/test_model_gpu.py -q > gpurun_out/r2_model.log 2>&1
tail -4 gpurun_out/r2_model.log
step 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2_prof.log 2>&1
tail -2 gpurun_out/r2_prof.log
find gpurun_out/prof_r2 -name "*stats*" | head
