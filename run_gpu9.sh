#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/r9_kernels.log 2>&1
tail -1 gpurun_out/r9_kernels.log
step 300 python vae-2_amd/tools/conv_bench.py > gpurun_out/r9_conv.log 2>&1
cat gpurun_out/r9_conv.log | grep -v amdgpu.ids
step 400 python bench.py --no-cpu-baseline > gpurun_out/r9_bench.log 2>&1
grep '^{' gpurun_out/r9_bench.log | cut -c1-200
grep '^{' gpurun_out/r9_bench.log | grep -o '"roofline.*'
step 400 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/r9_bench_nr.log 2>&1
grep '^{' gpurun_out/r9_bench_nr.log | cut -c1-200
