#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 600 python -m pytest tests/test_model_gpu.py -q > gpurun_out/r7_model.log 2>&1
tail -2 gpurun_out/r7_model.log
step 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r7_bench.log 2>&1
grep '^{' gpurun_out/r7_bench.log | cut -c1-250
