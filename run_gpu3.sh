#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/r3_kernels.log 2>&1
tail -3 gpurun_out/r3_kernels.log
step 600 python -m pytest tests/test_model_gpu.py -q > gpurun_out/r3_model.log 2>&1
tail -4 gpurun_out/r3_model.log
step 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3_bench.log 2>&1
tail -1 gpurun_out/r3_bench.log
step 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r3_prof.log 2>&1
